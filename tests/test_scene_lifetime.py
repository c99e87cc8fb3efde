"""rt_scene_destroy waits for its own scene's work only.

The header's threading contract: distinct scenes are independent and usable
from different host threads at once.  Destroying scene A must therefore not
stall behind scene B's long render on the same device (it used to call
hipDeviceSynchronize), and destroying a scene right after an asynchronous
rt_render_device on a caller stream must still be safe: the render finishes on
the scene's tables and buffers before they are released.  Scene memory is
stream-ordered (hipMallocAsync / hipFreeAsync on the scene's stream), since a
plain hipFree waits for the whole device (tools/free_probe.hip).
Ownership contract: SURVEY §8(b); the reference's singleton scene context,
/root/reference/src/scene/CudaSceneInitialization.cuh:302-308."""
import os
import threading
import time

import numpy as np
import pytest

from rtx import abi
from rtx.render import Renderer, camera_frame
from rtx.scene import load_scene

SCENES = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                      "real-time-ray-tracing-engine_amd", "scenes")

pytestmark = pytest.mark.gpu


def _long_frame(S, spp=1024):
    return camera_frame(S.camera_desc(image_width=1920, samples_per_pixel=spp, max_depth=8))


def test_destroy_does_not_wait_for_another_scenes_render():
    import gc
    import torch
    # earlier tests' garbage (pinned host tensors, streams) must not be freed
    # inside the timed window: torch's pinned-memory free (hipHostFree) waits
    # for the whole device, whatever the library does
    gc.collect()
    torch.cuda.synchronize()
    SB = load_scene(os.path.join(SCENES, "bouncing_seed42.json"))
    SA = load_scene(os.path.join(SCENES, "three_spheres.json"))
    fB = _long_frame(SB)
    fA = camera_frame(SA.camera_desc(image_width=64, samples_per_pixel=4, max_depth=4))
    dev = torch.device("cuda", 0)
    outB = torch.empty((fB.image_height, fB.image_width, 3), dtype=torch.float64, device=dev)
    outA = torch.empty((fA.image_height, fA.image_width, 3), dtype=torch.float64, device=dev)
    sB, sA = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    with Renderer(SB) as RB:
        RB.render_device(fB, outB.data_ptr(), sB.cuda_stream, seed=1, output=abi.RT_OUT_SUM,
                         accumulate=0)  # warm (buffers, tile order)
        sB.synchronize()
        t0 = time.perf_counter()
        RB.render_device(fB, outB.data_ptr(), sB.cuda_stream, seed=2, output=abi.RT_OUT_SUM,
                         accumulate=0)
        sB.synchronize()
        b_ms = (time.perf_counter() - t0) * 1e3
        assert b_ms > 50, b_ms  # long enough to tell the waits apart

        RA = Renderer(SA)
        RA.render_device(fA, outA.data_ptr(), sA.cuda_stream, seed=3, output=abi.RT_OUT_SUM,
                         accumulate=0)
        sA.synchronize()
        # B's long render in flight; A (idle) is destroyed from another thread
        gc.disable()
        RB.render_device(fB, outB.data_ptr(), sB.cuda_stream, seed=4, output=abi.RT_OUT_SUM,
                         accumulate=0)
        took = {}

        def destroy_a():
            t = time.perf_counter()
            RA.close()
            took["ms"] = (time.perf_counter() - t) * 1e3
        th = threading.Thread(target=destroy_a)
        try:
            t1 = time.perf_counter()
            th.start()
            th.join()
            joined_ms = (time.perf_counter() - t1) * 1e3
            b_done = not bool(sB.query())
        finally:
            gc.enable()
        sB.synchronize()
    # A's destroy returned while B's render was still running
    assert took["ms"] < 0.3 * b_ms, (took, b_ms)
    assert joined_ms < 0.5 * b_ms and b_done, (joined_ms, b_ms)


def test_destroy_right_after_an_async_launch_is_safe():
    """Destroy waits for the scene's own launch on the caller stream: the frame
    it leaves in the caller's buffer is the complete render (bit-identical to
    the same launch on a scene that stays alive)."""
    import torch
    S = load_scene(os.path.join(SCENES, "cornell_fog.json"))
    f = _long_frame(S, spp=256)
    dev = torch.device("cuda", 0)
    st = torch.cuda.Stream(dev)
    out = torch.full((f.image_height, f.image_width, 3), -1.0, dtype=torch.float64, device=dev)
    R = Renderer(S)
    R.render_device(f, out.data_ptr(), st.cuda_stream, seed=9, output=abi.RT_OUT_SUM, accumulate=0)
    t0 = time.perf_counter()
    R.close()  # must wait for the launch above, and only for it
    waited_ms = (time.perf_counter() - t0) * 1e3
    assert st.query(), "destroy returned before its scene's render finished"
    with Renderer(S) as R2:
        want = R2.render(f, seed=9, output=abi.RT_OUT_SUM)
    got = out.cpu().numpy()
    assert np.array_equal(np.isnan(got), np.isnan(want))
    assert np.array_equal(np.nan_to_num(got), np.nan_to_num(want))
    assert waited_ms > 1.0  # it did wait (the render takes tens of ms)


def test_scenes_on_many_streams_and_buffer_growth():
    """A scene used on several caller streams (and the null stream) in turn --
    each launch ordered after the previous one by a stream wait, as the
    threading contract asks (the launches of one scene share its work-unit
    counter), but with no host synchronisation between them -- with growing
    launches that reallocate its scratch and tile-order buffers while the
    earlier launches may still run: the frames equal a fresh scene's."""
    import torch
    S = load_scene(os.path.join(SCENES, "bouncing_seed42.json"))
    dev = torch.device("cuda", 0)
    streams = [torch.cuda.Stream(dev) for _ in range(3)] + [torch.cuda.default_stream(dev)]
    with Renderer(S) as R:
        outs = []
        prev = torch.cuda.current_stream(dev)
        for k, w in enumerate((64, 320, 960, 1920)):
            f = camera_frame(S.camera_desc(image_width=w, samples_per_pixel=64, max_depth=8))
            st = streams[k]
            with torch.cuda.stream(st):
                o = torch.empty((f.image_height, f.image_width, 3), dtype=torch.float64, device=dev)
            st.wait_stream(prev)
            R.render_device(f, o.data_ptr(), st.cuda_stream, seed=k, output=abi.RT_OUT_SUM,
                            accumulate=0)
            outs.append((f, k, o))
            prev = st
        torch.cuda.synchronize()
    with Renderer(S) as R2:
        for f, k, o in outs:
            want = R2.render(f, seed=k, output=abi.RT_OUT_SUM)
            assert np.array_equal(o.cpu().numpy(), want), f.image_width


def test_launches_on_unordered_streams_are_chained():
    """Launches of one scene on caller streams the caller did not order against
    each other (here: two streams, no waits, persistent-instance frames that
    share the scene's work-unit counter and scratch) run one after the other:
    the library orders each launch after the scene's previous one, so every
    frame equals a fresh scene's."""
    import torch
    S = load_scene(os.path.join(SCENES, "bouncing_seed42.json"))
    dev = torch.device("cuda", 0)
    streams = [torch.cuda.Stream(dev) for _ in range(2)]
    f = camera_frame(S.camera_desc(image_width=960, samples_per_pixel=64, max_depth=8))
    with Renderer(S) as R:
        outs = []
        for k in range(6):
            st = streams[k % 2]
            with torch.cuda.stream(st):
                o = torch.empty((f.image_height, f.image_width, 3), dtype=torch.float64, device=dev)
            R.render_device(f, o.data_ptr(), st.cuda_stream, seed=20 + k, output=abi.RT_OUT_SUM,
                            accumulate=0)
            outs.append(o)
        torch.cuda.synchronize()
    with Renderer(S) as R2:
        for k, o in enumerate(outs):
            assert np.array_equal(o.cpu().numpy(), R2.render(f, seed=20 + k, output=abi.RT_OUT_SUM)), k
