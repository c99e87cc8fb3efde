"""GPU parity: the HIP kernel (through the C ABI) vs the oracle's COUNTER mode.

Both sides draw the same Philox stream (DESIGN.md "RNG contract"), so per-pixel
results agree to floating-point rounding.  Bar (north star): |GPU - oracle| <=
1e-4 per channel on every pixel; pixel indexing is exact (checked through row
and stratum sharding identities).  The oracle itself is pinned bit-exact to the
real reference by tests/test_oracle.py.
"""
import json
import os

import numpy as np
import pytest

from rtx import abi
from rtx.render import Renderer, camera_frame
from rtx.scene import load_scene
import oracle_lib as O

pytestmark = pytest.mark.gpu

TOL = 1e-4  # per-channel absolute tolerance on scaled radiance (north star)
SCENES = os.path.join(O.ROOT, "real-time-ray-tracing-engine_amd", "scenes")
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def scene(name):
    if name.startswith("bouncing_") and name != "bouncing_seed42":
        with open(os.path.join(GOLD, "scene_variants.json")) as f:
            return load_scene(json.load(f)[name])
    return load_scene(os.path.join(SCENES, name + ".json"))


def compare(gpu, ref, tol=TOL):
    assert gpu.shape == ref.shape
    nan_g, nan_r = np.isnan(gpu), np.isnan(ref)
    assert np.array_equal(nan_g, nan_r), "NaN pattern differs"
    d = np.abs(np.where(nan_g, 0, gpu) - np.where(nan_r, 0, ref))
    bad = d > tol
    assert not bad.any(), "%d/%d channels differ by > %g (max %g)" % (
        bad.sum(), bad.size, tol, d.max())
    return float(d.max())


CASES = [
    # scene, width, spp, depth, seed, use_bvh override
    ("three_spheres", 64, 16, 8, 1, None),
    ("three_spheres", 61, 9, 8, 42, None),      # ragged tiles (61 x 34)
    ("cornell", 40, 16, 8, 1234, 0),
    ("cornell", 40, 16, 8, 1234, 1),            # lights as BVHNode (0.5/0.5 weights)
    ("cornell", 24, 4, 50, 7, 1),               # reference default depth 50
    ("cornell_fog", 48, 16, 8, 42, None),       # medium + Perlin + instances
    ("bouncing_seed42", 64, 4, 8, 42, None),    # 486 spheres, moving, defocus, checker
    ("bouncing_noglass", 48, 4, 8, 3, None),
]


@pytest.mark.parametrize("case", CASES, ids=lambda c: "%s_w%d_spp%d_d%d_s%d" % c[:5])
def test_gpu_matches_oracle_counter_mode(case):
    name, w, spp, depth, seed, bvh = case
    S = scene(name)
    if bvh is not None:
        S.use_bvh = bvh
    cam = S.camera_desc(image_width=w, samples_per_pixel=spp, max_depth=depth)
    f = camera_frame(cam)
    with Renderer(S) as R:
        gpu = R.render(f, seed=seed)
    ref = O.oracle_render(S, cam, O.MODE_COUNTER, seed)
    compare(gpu, ref)
    assert np.nanmean(gpu) > 0


def test_rows_and_strata_shard_exactly():
    """Pixel/stratum indexing: disjoint row batches and stratum ranges compose to
    the full render (the reference's 64-row batching, StaticCamera.cpp:235)."""
    S = scene("cornell_fog")
    cam = S.camera_desc(image_width=40, samples_per_pixel=16, max_depth=8)
    f = camera_frame(cam)
    with Renderer(S) as R:
        full = R.render(f, seed=5)
        top = R.render(f, seed=5, rows=(0, 9))
        bot = R.render(f, seed=5, rows=(9, f.image_height))
        # per-pixel sums are accumulated in LDS in completion order, so a different
        # tiling changes only the fp64 summation order
        np.testing.assert_allclose(np.concatenate([top, bot]), full, rtol=1e-12, atol=1e-15)
        s_full = R.render(f, seed=5, output=abi.RT_OUT_SUM)
        a = R.render(f, seed=5, samples=(0, 7), output=abi.RT_OUT_SUM)
        b = R.render(f, seed=5, samples=(7, 9), output=abi.RT_OUT_SUM)
        np.testing.assert_allclose(a + b, s_full, rtol=1e-12, atol=1e-12)
        np.testing.assert_allclose(s_full * f.pixel_samples_scale, full, rtol=1e-15, atol=0)


def test_full_hd_rows_match_oracle():
    """BASELINE config 2 geometry (1920x1080) on a band of rows the oracle can
    afford; every pixel of those rows within tolerance."""
    S = scene("three_spheres")
    cam = S.camera_desc(image_width=1920, samples_per_pixel=4, max_depth=8)
    f = camera_frame(cam)
    rows = (536, 548)
    with Renderer(S) as R:
        gpu = R.render(f, seed=11, rows=rows)
    ref = O.oracle_render(S, cam, O.MODE_COUNTER, 11, rows=rows)
    compare(gpu, ref)


# BASELINE configs at their own sample counts, on bands of full-width rows the
# threaded oracle can afford: C2 (spp 64), C3 (486-sphere BVH, defocus, motion
# blur, glass; spp 256), C4 (Cornell + fog + Perlin + lights; spp 1024).
BASELINE_BANDS = [("three_spheres", 64, (528, 544)), ("bouncing_seed42", 256, (516, 524)),
                  ("cornell_fog", 1024, (698, 702))]


@pytest.mark.parametrize("name,spp,rows", BASELINE_BANDS, ids=[b[0] for b in BASELINE_BANDS])
def test_baseline_spp_bands_match_oracle(name, spp, rows):
    S = scene(name)
    cam = S.camera_desc(image_width=1920, samples_per_pixel=spp, max_depth=8)
    f = camera_frame(cam)
    with Renderer(S) as R:
        gpu = R.render(f, seed=23, rows=rows)
    ref = O.oracle_render(S, cam, O.MODE_COUNTER, 23, rows=rows, threads=16)
    compare(gpu, ref)


def test_spp_not_square_scales_by_spp():
    """spp=10 traces 3x3 strata but scales by 1/10 (StaticCamera.cpp:74-76, 98)."""
    S = scene("three_spheres")
    cam = S.camera_desc(image_width=32, samples_per_pixel=10, max_depth=8)
    f = camera_frame(cam)
    assert f.sqrt_spp == 3 and f.pixel_samples_scale == 0.1
    with Renderer(S) as R:
        gpu = R.render(f, seed=1)
    compare(gpu, O.oracle_render(S, cam, O.MODE_COUNTER, 1))


def test_device_accumulation_and_to_bytes():
    torch = pytest.importorskip("torch")
    import ctypes as C
    from rtx.lib import load
    from rtx.ppm import to_bytes
    S = scene("three_spheres")
    cam = S.camera_desc(image_width=48, samples_per_pixel=9, max_depth=8)
    f = camera_frame(cam)
    buf = torch.zeros((f.image_height, f.image_width, 3), dtype=torch.float64, device="cuda:0")
    with Renderer(S) as R:
        stream = torch.cuda.current_stream().cuda_stream
        R.render_device(f, buf.data_ptr(), stream, seed=3, samples=(0, 4))
        R.render_device(f, buf.data_ptr(), stream, seed=3, samples=(4, 5))
        torch.cuda.synchronize()
        host = R.render(f, seed=3, output=abi.RT_OUT_SUM)
    np.testing.assert_allclose(buf.cpu().numpy(), host, rtol=1e-12, atol=1e-12)
    bytes_dev = torch.empty(buf.numel(), dtype=torch.uint8, device="cuda:0")
    L = load()
    assert L.rt_to_bytes_device(C.c_void_p(buf.data_ptr()), buf.numel() // 3,
                                f.pixel_samples_scale, C.c_void_p(bytes_dev.data_ptr()),
                                C.c_void_p(stream)) == 0
    torch.cuda.synchronize()
    want = to_bytes(buf.cpu().numpy() * f.pixel_samples_scale).reshape(-1)
    assert np.array_equal(bytes_dev.cpu().numpy(), want)


def test_stats_counters_are_consistent():
    S = scene("bouncing_seed42")
    cam = S.camera_desc(image_width=64, samples_per_pixel=4, max_depth=8)
    f = camera_frame(cam)
    with Renderer(S) as R:
        st = R.stats(f, seed=1)
        info = R.info()
    assert st["samples"] == f.image_width * f.image_height * 4
    assert st["samples"] <= st["segments"] <= 8 * st["samples"]
    assert st["node_visits"] > st["segments"]
    # every segment either misses (sky) or shades one hit
    assert 0 < st["shade_events"] <= st["segments"]
    assert info["n_spheres"] == 486 and info["bvh_depth"] < 30


def test_errors_are_reported_not_fatal():
    from rtx.lib import RtError
    S = scene("three_spheres")
    cam = S.camera_desc(image_width=16, samples_per_pixel=4, max_depth=8)
    f = camera_frame(cam)
    with Renderer(S) as R:
        with pytest.raises(RtError):
            R.render(f, seed=1, samples=(0, 5))   # beyond sqrt_spp^2 strata
        with pytest.raises(RtError):
            R.render(f, seed=1, rows=(3, 2))
        R.render(f, seed=1)                       # still usable afterwards


@pytest.mark.gpu
def test_render_device_is_ordered_with_torch_stream():
    """rt_render_device on the null stream is ordered with torch's default
    stream: zero_, render, accumulate, .cpu() need no explicit synchronize."""
    import torch
    S = scene("cornell")
    cam = S.camera_desc(image_width=48, samples_per_pixel=4, max_depth=6)
    f = camera_frame(cam)
    buf = torch.full((f.image_height, f.image_width, 3), 7.0, dtype=torch.float64, device="cuda")
    with Renderer(S) as R:
        for _ in range(3):
            buf.zero_()
            R.render_device(f, buf.data_ptr(), 0, seed=5, output=abi.RT_OUT_SUM, accumulate=1)
            R.render_device(f, buf.data_ptr(), 0, seed=5, output=abi.RT_OUT_SUM, accumulate=1)
            got = buf.cpu().numpy()  # syncs torch's stream only
        one = R.render(f, seed=5, output=abi.RT_OUT_SUM)
    np.testing.assert_allclose(got, 2 * one, rtol=1e-12, atol=1e-12)


@pytest.mark.gpu
def test_two_scenes_render_concurrently_from_two_threads():
    """Distinct rt_scene objects are independent (rt_api.h "Threading"): two host
    threads render two scenes at once and each matches its own oracle."""
    import threading
    jobs = [("cornell", 32, 9, 3), ("bouncing_seed42", 40, 4, 8)]
    out = {}

    def run(name, w, spp, seed):
        S = scene(name)
        cam = S.camera_desc(image_width=w, samples_per_pixel=spp, max_depth=6)
        with Renderer(S) as R:
            for _ in range(3):
                out[name] = (R.render(camera_frame(cam), seed=seed), S, cam, seed)

    th = [threading.Thread(target=run, args=j) for j in jobs]
    for t in th:
        t.start()
    for t in th:
        t.join()
    for name, (img, S, cam, seed) in out.items():
        compare(img, O.oracle_render(S, cam, O.MODE_COUNTER, seed))
