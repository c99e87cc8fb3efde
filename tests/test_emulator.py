"""The kernel's own per-path source (csrc/rt_path.h), compiled for the HOST by
g++ (tests/native, test-only), against the oracle's counter mode — for every
kernel feature instance.  Runs without a GPU; a failure here is a logic error
in the kernel source, while a GPU-only failure (tests/test_gpu_instances.py)
points at gfx950 code generation."""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

from rtx import abi
from rtx.render import camera_frame
from rtx.scene import load_scene
import oracle_lib as O
from test_gpu_instances import feature_scene

NATIVE = os.path.join(os.path.dirname(__file__), "native")


@pytest.fixture(scope="module")
def emu():
    subprocess.run(["make", "-s", "-C", NATIVE], check=True)
    L = C.CDLL(os.path.join(NATIVE, "build", "libemu.so"))
    L.emu_render.argtypes = [C.POINTER(abi.SceneDesc), C.POINTER(abi.Frame),
                             C.POINTER(abi.RenderParams), C.c_int, C.POINTER(C.c_double)]
    return L


@pytest.mark.parametrize("F", list(range(16)))
def test_kernel_source_on_host_matches_oracle(emu, F):
    S = load_scene(feature_scene(F))
    d = S.desc()
    cam = S.camera_desc(image_width=32, samples_per_pixel=9, max_depth=8)
    f = camera_frame(cam)
    p = abi.RenderParams()
    p.seed, p.sample_count, p.output = 77, -1, abi.RT_OUT_SCALED
    out = np.zeros((f.image_height, f.image_width, 3))
    assert emu.emu_render(C.byref(d), C.byref(f), C.byref(p), F,
                          out.ctypes.data_as(C.POINTER(C.c_double))) == 0
    ref = O.oracle_render(S, cam, O.MODE_COUNTER, 77)
    assert np.array_equal(np.isnan(out), np.isnan(ref))
    np.testing.assert_allclose(np.nan_to_num(out), np.nan_to_num(ref), rtol=0, atol=1e-12)
