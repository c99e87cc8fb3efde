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
