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
    # 1e-10: the kernel's sincos_2pi is within 1.4e-16 of sin/cos(2 pi u) while the
    # oracle calls libm on fl(2 pi u) (up to 4.4e-16 apart); bounces amplify that
    # to ~1e-12 on bright pixels.  Still eight orders below the GPU parity bar (1e-4).
    np.testing.assert_allclose(np.nan_to_num(out), np.nan_to_num(ref), rtol=0, atol=1e-10)


def test_sincos_2pi_accuracy(emu):
    """sincos_2pi (rt_path.h) against sin/cos(2 pi u) in long double, for u = k 2^-32
    (random k, both ends of the range, every quadrant boundary)."""
    rng = np.random.default_rng(5)
    k = np.concatenate([rng.integers(0, 2**32, size=200000), np.arange(4096), 2**32 - 1 - np.arange(4096),
                        np.arange(0, 2**32, 2**24),
                        (np.arange(1, 4)[:, None] * 2**30 + np.arange(-64, 64)[None, :]).ravel()])
    k = np.unique(k % 2**32)
    u = k.astype(np.float64) * 2.0**-32
    s, c = np.zeros_like(u), np.zeros_like(u)
    P = C.POINTER(C.c_double)
    emu.emu_sincos_2pi.argtypes = [P, C.c_int, P, P]
    emu.emu_sincos_2pi(u.ctypes.data_as(P), len(u), s.ctypes.data_as(P), c.ctypes.data_as(P))
    ang = 2 * np.longdouble("3.14159265358979323846264338327950288") * k.astype(np.longdouble) * np.longdouble(2.0)**-32
    assert float(np.abs(s - np.sin(ang)).max()) < 3e-16
    assert float(np.abs(c - np.cos(ang)).max()) < 3e-16
    assert np.all(np.abs(s) <= 1) and np.all(np.abs(c) <= 1)
    assert s[0] == 0.0 and c[0] == 1.0


def test_div_mk_equals_division(emu):
    """div_mk (rt_path.h: x * RN(1/b) plus one FMA correction, used for the sphere
    roots and ct/pi) returns the IEEE division's double, bit for bit, on random
    operands over the kernel's range, divisors with all-ones / all-zeros
    significands, pi, and the ray-tracing magnitudes (|d|^2 ~ 1, roots ~ 1e-3..1e3)."""
    rng = np.random.default_rng(11)
    n = 400000

    def rand_f64(lo_exp, hi_exp, m):
        sig = rng.uniform(1.0, 2.0, size=m)
        return sig * np.exp2(rng.integers(lo_exp, hi_exp, size=m).astype(np.float64))

    x = rand_f64(-900, 900, n) * rng.choice([-1.0, 1.0], size=n)
    b = rand_f64(-90, 90, n)
    ones = np.nextafter(np.exp2(rng.integers(-60, 60, size=20000).astype(np.float64) + 1), 0)  # 1.111...1 x 2^e
    pows = np.exp2(rng.integers(-60, 60, size=20000).astype(np.float64))
    xb = rand_f64(-30, 30, 40000 + 20000) * rng.choice([-1.0, 1.0], size=60000)
    bb = np.concatenate([ones, pows, np.full(20000, np.pi)])
    x = np.concatenate([x, xb, rng.uniform(-1, 1, 100000)])
    b = np.concatenate([b, bb, np.full(100000, np.pi)])
    q = np.zeros_like(x)
    P = C.POINTER(C.c_double)
    emu.emu_div_mk.argtypes = [P, P, C.c_int, P]
    emu.emu_div_mk(x.ctypes.data_as(P), b.ctypes.data_as(P), len(x), q.ctypes.data_as(P))
    want = x / b
    bad = q.view(np.uint64) != want.view(np.uint64)
    assert not bad.any(), (x[bad][:4], b[bad][:4], q[bad][:4], want[bad][:4])
