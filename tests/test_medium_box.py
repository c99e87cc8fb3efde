"""Box-boundary media: rt_path.h box_span (the six face distances as one slab
test, exact Plane::hit distances through one shared reciprocal per axis)
against the general boundary_span and against the reference's own
ConstantMedium boundary queries (ConstantMedium.cpp:28-32 over make_box under
RotateY / Translate, PlaneUtility.hpp:11-39, Plane.cpp:76-113).

Golden: tests/golden/ref_medium_box.npz, from oracle/_ref by
tests/golden/make_medium_kats.py, on the 120k deterministic rays of
tests/medium_rays.py (edge, corner, grazing, axis-parallel, inside, on-face and
scaled rays besides random ones).  Bit-exact: every t box_span reports is the
reference's double, every span it decides is the reference's decision, and
boundary_span (the fallback for the rays box_span defers) matches the
reference on every ray.  The host build is tests/native's emulator (the kernel
source under g++); the device build is tests/native/rt_devcheck.hip (gfx950).
"""
import ctypes as C
import os
import subprocess
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(ROOT, "real-time-ray-tracing-engine_amd"))
sys.path.insert(0, HERE)

from rtx import abi  # noqa: E402
from rtx.scene import load_scene  # noqa: E402
import medium_rays  # noqa: E402

GOLDEN = os.path.join(HERE, "golden", "ref_medium_box.npz")
NATIVE = os.path.join(HERE, "native", "build")
SCENES = os.path.join(ROOT, "real-time-ray-tracing-engine_amd", "scenes")
P = C.POINTER(C.c_double)


def _golden():
    g = np.load(GOLDEN)
    rays = medium_rays.make_rays(int(g["n_rays"]), int(g["seed"]))
    return g, rays


def _fog_desc():
    S = load_scene(os.path.join(SCENES, "cornell_fog.json"))
    return S, S.desc()


def _spans(fn, d, rays, m=0):
    n = len(rays)
    out = np.zeros((n, 6))
    rays = np.ascontiguousarray(rays)
    rc = fn(C.addressof(d), m, rays.ctypes.data_as(P), n, out.ctypes.data_as(P))
    assert rc == 0, rc
    return out


def _emu():
    L = C.CDLL(os.path.join(NATIVE, "libemu.so"))
    L.emu_medium_spans.argtypes = [C.c_void_p, C.c_int, P, C.c_int, P]
    return L.emu_medium_spans


def check_against_golden(out, g):
    """out: emu/devcheck rows (box code, t1, t2, general flag, t1, t2)."""
    ref_span = (g["hit1"] == 1) & (g["hit2"] == 1)
    gen = out[:, 3] == 1
    # boundary_span == the reference on every ray (its spans and their t's)
    assert np.array_equal(gen, ref_span)
    assert np.array_equal(out[gen, 4], g["t1"][gen]) and np.array_equal(out[gen, 5], g["t2"][gen])
    rc = out[:, 0]
    assert set(np.unique(rc)) <= {-1.0, 0.0, 1.0}  # the fog medium is a box
    dec = rc >= 0
    # box_span's decisions are the reference's, its t's the reference's doubles
    assert np.array_equal(rc[dec] == 1, ref_span[dec])
    b = rc == 1
    assert np.array_equal(out[b, 1], g["t1"][b]) and np.array_equal(out[b, 2], g["t2"][b])
    return rc


def test_box_span_matches_reference_on_the_host():
    g, rays = _golden()
    S, d = _fog_desc()
    out = _spans(_emu(), d, rays)
    rc = check_against_golden(out, g)
    fam = np.arange(len(rays)) % 8
    # random rays, rays from inside / on a face, scaled rays: box_span decides
    # (almost) all; only edge, corner, grazing and near-parallel rays defer
    for f in (0, 4, 5, 6):
        assert (rc[fam == f] < 0).mean() == 0.0, f
    assert (rc >= 0).mean() > 0.7
    # deferred rays exist in the adversarial families (the fallback is exercised)
    assert (rc[np.isin(fam, (1, 2, 3, 7))] < 0).sum() > 1000


def test_non_box_boundaries_keep_the_general_scan():
    import json
    # a medium whose boundary is a sphere: not a box (code -2), boundary_span only
    with open(os.path.join(SCENES, "cornell_fog.json")) as f:
        doc = json.load(f)
    for o in doc["world"]:
        if o["type"] == "constant_medium":
            o["boundary"] = {"type": "sphere", "center": [300, 150, 300], "radius": 100,
                             "material": "white"}
    S2 = load_scene(doc)
    d2 = S2.desc()
    rays = medium_rays.make_rays(2000, 11)
    out = _spans(_emu(), d2, rays)
    assert np.all(out[:, 0] == -2)
    # a box made of 5 faces (one removed) is not a box either
    with open(os.path.join(SCENES, "cornell_fog.json")) as f:
        doc = json.load(f)
    faces = [{"type": "quad", "Q": [0, 0, 0], "u": [165, 0, 0], "v": [0, 330, 0], "material": "white"},
             {"type": "quad", "Q": [0, 0, 165], "u": [165, 0, 0], "v": [0, 330, 0], "material": "white"},
             {"type": "quad", "Q": [0, 0, 0], "u": [0, 0, 165], "v": [0, 330, 0], "material": "white"},
             {"type": "quad", "Q": [165, 0, 0], "u": [0, 0, 165], "v": [0, 330, 0], "material": "white"},
             {"type": "quad", "Q": [0, 0, 0], "u": [165, 0, 0], "v": [0, 0, 165], "material": "white"}]
    for o in doc["world"]:
        if o["type"] == "constant_medium":
            o["boundary"] = {"type": "list", "objects": faces}
    out = _spans(_emu(), load_scene(doc).desc(), rays)
    assert np.all(out[:, 0] == -2)
    # the same five plus the top face: a box again, and box_span == boundary_span
    faces.append({"type": "quad", "Q": [0, 330, 0], "u": [165, 0, 0], "v": [0, 0, 165],
                  "material": "white"})
    for o in doc["world"]:
        if o["type"] == "constant_medium":
            o["boundary"] = {"type": "list", "objects": faces}
    out = _spans(_emu(), load_scene(doc).desc(), rays)
    assert set(np.unique(out[:, 0])) <= {-1.0, 0.0, 1.0}
    b = out[:, 0] == 1
    assert b.sum() > 100
    assert np.array_equal(out[b, 1:3], out[b, 4:6])
    dec = out[:, 0] >= 0
    assert np.array_equal(out[dec, 0] == 1, out[dec, 3] == 1)


@pytest.mark.skipif(not os.path.exists("/root/reference/src"), reason="needs the reference tree")
def test_medium_golden_regenerates_identically(tmp_path):
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "ref"], check=True)
    subprocess.run([sys.executable, os.path.join(HERE, "golden", "make_medium_kats.py"), str(tmp_path)],
                   check=True)
    a, b = np.load(GOLDEN), np.load(os.path.join(tmp_path, "ref_medium_box.npz"))
    for k in a.files:
        assert np.array_equal(a[k], b[k]), k


@pytest.mark.gpu
def test_box_span_matches_reference_on_the_device():
    L = C.CDLL(os.path.join(NATIVE, "libdevcheck.so"))
    L.devcheck_medium_spans.argtypes = [C.c_void_p, C.c_int, P, C.c_int, P]
    g, rays = _golden()
    S, d = _fog_desc()
    dev = _spans(L.devcheck_medium_spans, d, rays)
    check_against_golden(dev, g)
    host = _spans(_emu(), d, rays)
    assert np.array_equal(dev, host)  # device == host build, deferrals included
