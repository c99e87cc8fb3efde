"""Progressive accumulation: the reference's interactive camera without the window.

DynamicCamera (DynamicCamera.cpp:96-200 CPU, 455-530 GPU) renders ONE stratum
of every pixel per frame, adds it to an accumulation buffer, and displays
accumulation * (1 / max(1, samples_taken)) through write_color (:284-300).  It
stops adding samples once every stratum of the ⌊√spp⌋² grid has been traced
(:111, :468) and clears the buffer when the camera moves (:269-276).

Here a frame is one rt_render_device launch over stratum k
(sample_begin = k, sample_count = n) that adds into a device-resident fp64
accumulator; rt_to_bytes_device quantises on the device.  The random stream is
keyed by the global stratum index, so after all strata the accumulator holds
exactly the sample sum of the static render with the same seed (tests check
this).

The render function is pluggable (as in rtx.dist) so the bookkeeping runs
on the CPU with the oracle in tests/; on a GPU use `for_renderer`.
"""
import ctypes as C

from . import abi
from .lib import check, load


class ProgressiveRenderer:
    """render_fn(frame, acc, seed, (first_stratum, count)) must ADD raw sample
    sums of those strata into `acc` (a [H, W, 3] float64 tensor)."""

    def __init__(self, render_fn, frame, acc, seed=0):
        self.render_fn = render_fn
        self.frame = frame
        self.acc = acc
        self.seed = seed
        self.samples_taken = 0

    @property
    def total_strata(self):
        return self.frame.sqrt_spp * self.frame.sqrt_spp

    @property
    def converged(self):
        return self.samples_taken >= self.total_strata  # DynamicCamera.cpp:111

    def step(self, n=1):
        """Trace the next n strata (one per frame in the reference); returns the
        number actually traced (0 once converged)."""
        n = max(0, min(n, self.total_strata - self.samples_taken))
        if n:
            self.render_fn(self.frame, self.acc, self.seed, (self.samples_taken, n))
            self.samples_taken += n
        return n

    @property
    def scale(self):
        return 1.0 / max(1, self.samples_taken)  # DynamicCamera.cpp:287

    def image(self):
        """The displayed radiance: accumulation x 1/max(1, samples_taken)."""
        return self.acc * self.scale

    def reset(self, frame=None):
        """Camera moved (DynamicCamera.cpp:269-276): clear and restart."""
        if frame is not None:
            self.frame = frame
        self.acc.zero_()
        self.samples_taken = 0


class AdaptiveFrames:
    """DynamicCamera's frame-rate controller (DynamicCamera.cpp:181-195) on this
    renderer's per-frame knob.  The reference measures frames per second once a
    second and doubles its tile size (16 -> 64, DynamicCamera.hpp:32-34) when
    fps > 30, halves it when fps < 15, and stops adapting once converged.  Its
    tile size only changes how a frame's work is scheduled; here a frame is one
    launch, and the knob that trades frame rate for progress is the number of
    strata traced per frame: doubled above 30 fps, halved below 15, within
    [min_strata, max_strata] (default 1..4, the reference's 16..64 ratio).  The
    converged image does not depend on it (every stratum is traced once).

        ctl = AdaptiveFrames(pr)
        while not pr.converged:
            ctl.frame()          # traces ctl.strata strata, adapts once a second
    """

    def __init__(self, pr, min_strata=1, max_strata=4, clock=None, window_s=1.0):
        import time
        self.pr = pr
        self.min_strata, self.max_strata = int(min_strata), int(max_strata)
        self.strata = self.min_strata
        self.clock = clock or time.perf_counter
        self.window_s = window_s
        self.fps = 0.0
        self._frames = 0
        self._t0 = self.clock()

    def frame(self):
        """One displayed frame: trace `strata` strata (0 once converged), then
        update the frame-rate estimate and adapt (DynamicCamera.cpp:181-195)."""
        n = self.pr.step(self.strata)
        self._frames += 1
        now = self.clock()
        elapsed = now - self._t0
        if elapsed >= self.window_s:
            self.fps = self._frames / elapsed
            self._frames = 0
            self._t0 = now
            converged = self.pr.converged
            if not converged and self.fps > 30.0 and self.strata < self.max_strata:
                self.strata = min(self.strata * 2, self.max_strata)
            elif not converged and self.fps < 15.0 and self.strata > self.min_strata:
                self.strata = max(self.strata // 2, self.min_strata)
        return n


def for_renderer(renderer, frame, seed=0, device=None, stream=None):
    """A ProgressiveRenderer over librtx_hip on a torch CUDA device."""
    import torch
    dev = torch.device("cuda", renderer.device if device is None else device)
    acc = torch.zeros((frame.image_height, frame.image_width, 3), dtype=torch.float64, device=dev)
    st = stream if stream is not None else torch.cuda.current_stream(dev)

    def render_fn(fr, a, sd, strata):
        renderer.render_device(fr, a.data_ptr(), st.cuda_stream, seed=sd, samples=strata,
                               output=abi.RT_OUT_SUM, accumulate=1)

    pr = ProgressiveRenderer(render_fn, frame, acc, seed)
    pr.stream = st
    return pr


def frame_bytes(pr, out=None):
    """write_color bytes of the displayed image, quantised on the device
    (rt_to_bytes_device); returns a [H, W, 3] uint8 CUDA tensor."""
    import torch
    if out is None:
        out = torch.empty(pr.acc.shape, dtype=torch.uint8, device=pr.acc.device)
    stream = getattr(pr, "stream", None) or torch.cuda.current_stream(pr.acc.device)
    check(load().rt_to_bytes_device(C.c_void_p(pr.acc.data_ptr()), pr.acc.numel() // 3,
                                    C.c_double(pr.scale), C.c_void_p(out.data_ptr()),
                                    C.c_void_p(stream.cuda_stream)))
    return out


_hip_rt = None


def _hip():
    """The HIP runtime torch loaded (one runtime per process, rtx/lib.py)."""
    global _hip_rt
    if _hip_rt is None:
        import os
        import torch
        L = C.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
        L.hipMemcpyAsync.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_void_p]
        L.hipMemcpyAsync.restype = C.c_int
        _hip_rt = L
    return _hip_rt


class DisplayPipeline:
    """Progressive frames to host memory without waiting for each frame's copy.

    The reference's GPU loop renders a frame, copies the whole fp64
    accumulator back and converts it on the host before the next frame starts
    (DynamicCamera.cpp:455-530).  Here frame k is quantised on the device
    (rt_to_bytes_device, 6.2 MB at 1080p) and copied to pinned host memory on a
    copy stream while frame k+1 renders; `present()` hands the viewer the bytes
    of the newest frame whose copy has finished -- one frame behind the render,
    so a frame costs max(render + quantise, copy) instead of their sum.  The
    bytes of every frame are the same as the synchronous loop's
    (tests/test_progressive.py).

        pipe = DisplayPipeline(for_renderer(R, frame, seed=5))
        while not pipe.pr.converged:
            pipe.frame()                 # issue frame k (render, bytes, copy)
            img = pipe.present()         # bytes of frame k-1 (None at first)
    """

    def __init__(self, pr, depth=2):
        import torch
        self.pr = pr
        dev = pr.acc.device
        self.stream = getattr(pr, "stream", None) or torch.cuda.current_stream(dev)
        # one copy stream: the copy split over 2 / 4 streams measured 2x / 4x
        # slower (1080p C2: 0.93 / 2.0 ms a frame against 0.47; the device's
        # few hardware queues, GPU_MAX_HW_QUEUES 4, are shared by then)
        self.copy_stream = torch.cuda.Stream(dev)
        self.depth = max(2, int(depth))
        shape = pr.acc.shape
        self.dbytes = [torch.empty(shape, dtype=torch.uint8, device=dev) for _ in range(self.depth)]
        self.hbytes = [torch.empty(shape, dtype=torch.uint8, pin_memory=True) for _ in range(self.depth)]
        # per slot, created once: bytes ready on the render stream, copy done
        self.ready = [torch.cuda.Event() for _ in range(self.depth)]
        self.copied = [torch.cuda.Event() for _ in range(self.depth)]
        self.used = [False] * self.depth   # the slot holds a frame
        self.synced = [False] * self.depth # ... whose copy the host has seen finish
        self.nbytes = self.dbytes[0].numel()
        self.samples = [0] * self.depth    # strata accumulated in the slot's frame
        self.issued = 0                    # frames issued

    def frame(self, n=1):
        """Issue the next frame: n strata added on the render stream, its bytes
        quantised there and copied to the host on the copy stream.  Returns the
        strata traced (0 once converged: the frame re-sends the final image)."""
        b = self.issued % self.depth
        if self.used[b] and not self.synced[b]:
            self.copied[b].synchronize()             # the viewer's copy of this slot is free
        self.synced[b] = False
        traced = self.pr.step(n)
        frame_bytes(self.pr, self.dbytes[b])
        self.ready[b].record(self.stream)
        self.copy_stream.wait_event(self.ready[b])
        # the D2H copy on the copy stream: one runtime call (torch's copy_
        # under a stream context costs several times that in host time)
        rc = _hip().hipMemcpyAsync(C.c_void_p(self.hbytes[b].data_ptr()),
                                   C.c_void_p(self.dbytes[b].data_ptr()),
                                   C.c_size_t(self.nbytes), 2,  # hipMemcpyDeviceToHost
                                   C.c_void_p(self.copy_stream.cuda_stream))
        if rc != 0:
            raise RuntimeError("hipMemcpyAsync failed (%d)" % rc)
        self.copied[b].record(self.copy_stream)
        self.used[b] = True
        self.samples[b] = self.pr.samples_taken
        self.issued += 1
        return traced

    def present(self, lag=1):
        """Host bytes [H, W, 3] (uint8) of the frame issued `lag` frames before
        the newest (default: the previous one, whose copy overlapped the newest
        frame's render), after its copy has finished; None if there is none."""
        k = self.issued - 1 - int(lag)
        if k < 0 or lag >= self.depth:
            return None
        b = k % self.depth
        if not self.synced[b]:
            self.copied[b].synchronize()
            self.synced[b] = True
        return self.hbytes[b]

    def flush(self):
        """Bytes of the newest frame (waits for its copy)."""
        return self.present(lag=0)
