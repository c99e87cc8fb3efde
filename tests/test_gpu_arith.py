"""The kernel's shortened fp64 sequences (rt_path.h), compiled for gfx950 and run
on the GPU, against the full IEEE operations on the same device, bit for bit:

* sqrt_n(x) — the compiler's correctly rounded sqrt lowering without its
  sub-2^-767 input scaling — on every input range the kernel feeds it
  (u = k 2^-32, 1 - u, 1 - x^2, squared lengths, 0, +inf, negatives, NaN);
* div_mk(x, b, 1/b) — the Markstein quotient from a shared reciprocal — on
  random operands, divisors with all-ones / power-of-two significands, and pi;
* rcp_n(x) — the division lowering for 1/x without scaling and fixup — on
  [2^-600, 2^600], all-ones significands, the unit range, and +inf;
* sincos_2pi with its polynomial constants materialised at their use (SGPR and
  VGPR forms, RT_KCONST) against the form that holds them, and against the
  host build (tests/native emulator) of the same function.

tests/native/build/libdevcheck.so is test-only (tests/native/Makefile).
"""
import ctypes as C
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

LIB = os.path.join(os.path.dirname(__file__), "native", "build", "libdevcheck.so")


@pytest.fixture(scope="module")
def dev():
    assert os.path.exists(LIB), "build tests/native first (make -C tests/native)"
    L = C.CDLL(LIB)
    P = C.POINTER(C.c_double)
    L.devcheck_arith.argtypes = [P, P, C.c_int, P, P, P, P]
    L.devcheck_arith.restype = C.c_int
    return L


def run(dev, x, b):
    x = np.ascontiguousarray(x, np.float64)
    b = np.ascontiguousarray(b, np.float64)
    outs = [np.zeros_like(x) for _ in range(4)]
    P = C.POINTER(C.c_double)
    rc = dev.devcheck_arith(x.ctypes.data_as(P), b.ctypes.data_as(P), len(x), *[o.ctypes.data_as(P) for o in outs])
    assert rc == 0, rc
    return outs


def same_bits(a, b):
    return (a.view(np.uint64) == b.view(np.uint64)) | (np.isnan(a) & np.isnan(b))


def test_sqrt_n_equals_sqrt_on_device(dev):
    rng = np.random.default_rng(3)
    k = rng.integers(0, 2**32, size=1_000_000).astype(np.float64)
    u = k * 2.0**-32
    z = 1.0 - 2.0 * u
    c = rng.uniform(-1, 1, 500_000)
    sig = rng.uniform(1.0, 2.0, 1_000_000) * np.exp2(rng.integers(-760, 1000, 1_000_000).astype(np.float64))
    special = np.array([0.0, -0.0, np.inf, -1.0, -np.inf, np.nan, 2.0**-767, 2.0**-766, 1.0, 2.0**-32,
                        1 - 2.0**-32, np.nextafter(1.0, 0), 2.0**-53, 2.0**-106])
    x = np.concatenate([u, 1.0 - u, np.maximum(0.0, 1.0 - z * z), 1.0 - c * c, np.abs(1.0 - c * c * 0.75),
                        sig, special])
    sq_n, sq, _, _ = run(dev, x, np.ones_like(x))
    ok = same_bits(sq_n, sq)
    assert ok.all(), (x[~ok][:4], sq_n[~ok][:4], sq[~ok][:4])


def test_div_mk_equals_division_on_device(dev):
    rng = np.random.default_rng(4)
    n = 1_000_000
    x = rng.uniform(1.0, 2.0, n) * np.exp2(rng.integers(-900, 900, n).astype(np.float64)) * rng.choice([-1.0, 1.0], n)
    b = rng.uniform(1.0, 2.0, n) * np.exp2(rng.integers(-90, 90, n).astype(np.float64))
    ones = np.nextafter(np.exp2(rng.integers(-60, 60, 100_000).astype(np.float64) + 1), 0)
    pows = np.exp2(rng.integers(-60, 60, 100_000).astype(np.float64))
    xs = rng.uniform(-1e3, 1e3, 300_000)
    bs = np.concatenate([ones, pows, np.full(100_000, np.pi)])
    x = np.concatenate([x, xs])
    b = np.concatenate([b, bs])
    _, _, dq, dv = run(dev, x, b)
    ok = same_bits(dq, dv)
    assert ok.all(), (x[~ok][:4], b[~ok][:4], dq[~ok][:4], dv[~ok][:4])


def test_rcp_n_equals_reciprocal_on_device(dev):
    rng = np.random.default_rng(6)
    n = 1_000_000
    x = rng.uniform(1.0, 2.0, n) * np.exp2(rng.integers(-600, 601, n).astype(np.float64))
    ones = np.nextafter(np.exp2(rng.integers(-600, 600, 100_000).astype(np.float64) + 1), 0)
    unit = rng.uniform(1e-8, 4.0, 300_000)
    x = np.concatenate([x, ones, unit, [np.inf, 1.0, 1e-8, 2.0**512, 1.3407807929942596e154]])
    _, _, dq, dv = run(dev, x, np.zeros_like(x))
    ok = same_bits(dq, dv)
    assert ok.all(), (x[~ok][:4], dq[~ok][:4], dv[~ok][:4])


def test_sincos_constant_forms_identical_on_device(dev):
    dev.devcheck_sincos.argtypes = [C.POINTER(C.c_double), C.c_int, C.POINTER(C.c_double)]
    dev.devcheck_sincos.restype = C.c_int
    rng = np.random.default_rng(5)
    u = np.concatenate([rng.integers(0, 2**32, 1_000_000).astype(np.float64) * 2.0**-32,
                        np.arange(0, 4097, dtype=np.float64) / 4096.0 * (1 - 2.0**-32),
                        np.array([0.0, 0.125, 0.25, 0.375, 0.5, 0.75, 1 - 2.0**-32])])
    out = np.zeros(6 * len(u))
    P = C.POINTER(C.c_double)
    rc = dev.devcheck_sincos(u.ctypes.data_as(P), len(u), out.ctypes.data_as(P))
    assert rc == 0, rc
    s0, c0, s1, c1, s2, c2 = out.reshape(6, len(u))
    for a, b in ((s1, s0), (c1, c0), (s2, s0), (c2, c0)):
        ok = same_bits(a, b)
        assert ok.all(), (u[~ok][:4], a[~ok][:4], b[~ok][:4])
    emu = os.path.join(os.path.dirname(__file__), "native", "build", "libemu.so")
    E = C.CDLL(emu)
    E.emu_sincos_2pi.argtypes = [P, C.c_int, P, P]
    hs, hc = np.zeros_like(u), np.zeros_like(u)
    E.emu_sincos_2pi(u.ctypes.data_as(P), len(u), hs.ctypes.data_as(P), hc.ctypes.data_as(P))
    assert same_bits(s0, hs).all() and same_bits(c0, hc).all()
