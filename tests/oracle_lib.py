"""ctypes bindings of the oracle (oracle/build/liboracle.so) and of the reference
bridge (oracle/_ref/libref.so).  TEST INFRASTRUCTURE: imported only by tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg."""
import ctypes as C
import os
import subprocess

import numpy as np

from rtx import abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
ORACLE_SO = os.path.join(ORACLE_DIR, "build", "liboracle.so")
REF_SO = os.path.join(ORACLE_DIR, "_ref", "libref.so")

MODE_MT, MODE_COUNTER = 0, 1

_oracle = None
_ref = None


def build_oracle():
    subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)


def oracle():
    global _oracle
    if _oracle is None:
        if not os.path.exists(ORACLE_SO):
            build_oracle()
        L = C.CDLL(ORACLE_SO)
        P = C.POINTER
        L.oracle_render.argtypes = [P(abi.SceneDesc), P(abi.CameraDesc), C.c_int, C.c_uint64,
                                    C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                    C.c_int, P(C.c_double)]
        L.oracle_render.restype = C.c_int
        L.oracle_camera_setup.argtypes = [P(abi.CameraDesc), P(abi.Frame)]
        L.oracle_philox.argtypes = [P(C.c_uint32), P(C.c_uint32), P(C.c_uint32)]
        L.oracle_u01x4.argtypes = [C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                                   P(C.c_double)]
        L.oracle_to_byte.argtypes = [C.c_double]
        L.oracle_to_byte.restype = C.c_ubyte
        L.oracle_object_hit.argtypes = [P(abi.SceneDesc), C.c_int, P(C.c_double), C.c_double,
                                        C.c_double, P(C.c_double)]
        L.oracle_object_pdf.argtypes = [P(abi.SceneDesc), C.c_int, P(C.c_double), P(C.c_double)]
        L.oracle_object_pdf.restype = C.c_double
        L.oracle_texture_value.argtypes = [P(abi.SceneDesc), C.c_int, C.c_double, C.c_double,
                                           P(C.c_double), P(C.c_double)]
        _oracle = L
    return _oracle


def ref_available():
    return os.path.exists(REF_SO)


def ref():
    global _ref
    if _ref is None:
        L = C.CDLL(REF_SO)
        P = C.POINTER
        L.ref_render.argtypes = [P(abi.SceneDesc), P(abi.CameraDesc), C.c_uint32, C.c_int,
                                 P(C.c_double)]
        L.ref_render_static.argtypes = [P(abi.SceneDesc), P(abi.CameraDesc), C.c_uint32, C.c_int,
                                        C.c_int, C.c_char_p]
        L.ref_camera_setup.argtypes = [P(abi.CameraDesc), P(abi.Frame)]
        L.ref_object_hit.argtypes = [P(abi.SceneDesc), C.c_int, P(C.c_double), C.c_double,
                                     C.c_double, P(C.c_double)]
        L.ref_object_pdf.argtypes = [P(abi.SceneDesc), C.c_int, P(C.c_double), P(C.c_double)]
        L.ref_object_pdf.restype = C.c_double
        L.ref_object_random.argtypes = [P(abi.SceneDesc), C.c_int, P(C.c_double), C.c_uint32,
                                        P(C.c_double)]
        L.ref_texture_value.argtypes = [P(abi.SceneDesc), C.c_int, C.c_double, C.c_double,
                                        P(C.c_double), P(C.c_double)]
        L.ref_to_byte.argtypes = [C.c_double]
        L.ref_to_byte.restype = C.c_ubyte
        _ref = L
    return _ref


def dptr(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


def image_height(cam):
    return max(1, int(cam.image_width / cam.aspect_ratio))


def oracle_render(scene, cam, mode, seed, use_bvh=None, rows=(0, 0), samples=(0, -1),
                  output=abi.RT_OUT_SCALED, threads=0):
    d = scene.desc()
    h = image_height(cam)
    r0, r1 = rows
    if r1 <= r0:
        r0, r1 = 0, h
    out = np.zeros((r1 - r0, cam.image_width, 3), dtype=np.float64)
    bvh = scene.use_bvh if use_bvh is None else use_bvh
    rc = oracle().oracle_render(C.byref(d), C.byref(cam), mode, seed, int(bvh), r0, r1,
                                samples[0], samples[1], output, threads, dptr(out))
    if rc != 0:
        raise RuntimeError("oracle_render failed")
    return out


def ref_render(scene, cam, seed, use_bvh=None):
    d = scene.desc()
    h = image_height(cam)
    out = np.zeros((h, cam.image_width, 3), dtype=np.float64)
    bvh = scene.use_bvh if use_bvh is None else use_bvh
    ref().ref_render(C.byref(d), C.byref(cam), seed, int(bvh), dptr(out))
    return out


def ref_binding_roundtrip(scene):
    """Scene -> reference objects -> INTEGRATION.md's binding (oracle/ref_binding.hpp)
    -> a new SceneDescription built from the binding's tables."""
    from rtx.scene import SceneDescription
    d = scene.desc()
    out = abi.SceneDesc()
    L = ref()
    L.ref_binding_roundtrip.argtypes = [C.POINTER(abi.SceneDesc), C.POINTER(abi.SceneDesc)]
    assert L.ref_binding_roundtrip(C.byref(d), C.byref(out)) == 0
    R = SceneDescription()
    R.textures = [abi.TextureDesc.from_buffer_copy(out.textures[k]) for k in range(out.n_textures)]
    R.perlin = [abi.PerlinDesc.from_buffer_copy(out.perlin[k]) for k in range(out.n_perlin)]
    R.materials = [abi.MaterialDesc.from_buffer_copy(out.materials[k]) for k in range(out.n_materials)]
    R.objects = [abi.ObjectDesc.from_buffer_copy(out.objects[k]) for k in range(out.n_objects)]
    R.children = [int(out.children[k]) for k in range(out.n_children)]
    R.world, R.lights, R.use_bvh = out.world, out.lights, out.use_bvh
    R.camera = scene.camera
    return R


def ref_trace_parallel(scene, cam, threads, use_bvh=None):
    """Reference code, -p decomposition over `threads` host threads (CPU baseline)."""
    d = scene.desc()
    h = image_height(cam)
    out = np.zeros((h, cam.image_width, 3), dtype=np.float64)
    bvh = scene.use_bvh if use_bvh is None else use_bvh
    L = ref()
    L.ref_trace_parallel.argtypes = [C.POINTER(abi.SceneDesc), C.POINTER(abi.CameraDesc), C.c_int,
                                     C.c_int, C.POINTER(C.c_double)]
    L.ref_trace_parallel.restype = C.c_longlong
    n = L.ref_trace_parallel(C.byref(d), C.byref(cam), int(bvh), int(threads), dptr(out))
    return n, out


def ref_trace_pool(scene, cam, threads, use_bvh=None):
    """Reference code, render_cpu's -p loop on the reference's ThreadPool with
    `threads` workers (CPU baseline sized to the host's CPU quota)."""
    d = scene.desc()
    h = image_height(cam)
    out = np.zeros((h, cam.image_width, 3), dtype=np.float64)
    bvh = scene.use_bvh if use_bvh is None else use_bvh
    L = ref()
    L.ref_trace_pool.argtypes = [C.POINTER(abi.SceneDesc), C.POINTER(abi.CameraDesc), C.c_int,
                                 C.c_int, C.POINTER(C.c_double)]
    L.ref_trace_pool.restype = C.c_longlong
    n = L.ref_trace_pool(C.byref(d), C.byref(cam), int(bvh), int(threads), dptr(out))
    return n, out


def ref_sample_batch(kind, seed, n):
    L = ref()
    L.ref_sample_batch.argtypes = [C.c_int, C.c_uint32, C.c_int, C.POINTER(C.c_double)]
    out = np.zeros((n, 3))
    assert L.ref_sample_batch(kind, seed, n, dptr(out)) == 0
    return out


def ref_light_batch(scene, org, seed, n, use_bvh=None):
    L = ref()
    L.ref_light_batch.argtypes = [C.POINTER(abi.SceneDesc), C.c_int, C.POINTER(C.c_double),
                                  C.c_uint32, C.c_int, C.POINTER(C.c_double)]
    d = scene.desc()
    o = np.ascontiguousarray(org, dtype=np.float64)
    out = np.zeros((n, 3))
    bvh = scene.use_bvh if use_bvh is None else use_bvh
    assert L.ref_light_batch(C.byref(d), int(bvh), dptr(o), seed, n, dptr(out)) == 0
    return out


def oracle_ctr_sample_batch(kind, seed, n):
    L = oracle()
    L.oracle_ctr_sample_batch.argtypes = [C.c_int, C.c_uint64, C.c_int, C.POINTER(C.c_double)]
    out = np.zeros((n, 3))
    assert L.oracle_ctr_sample_batch(kind, seed, n, dptr(out)) == 0
    return out


def oracle_ctr_light_batch(scene, org, seed, n, use_bvh=None):
    L = oracle()
    L.oracle_ctr_light_batch.argtypes = [C.POINTER(abi.SceneDesc), C.c_int, C.POINTER(C.c_double),
                                         C.c_uint64, C.c_int, C.POINTER(C.c_double)]
    d = scene.desc()
    o = np.ascontiguousarray(org, dtype=np.float64)
    out = np.zeros((n, 3))
    bvh = scene.use_bvh if use_bvh is None else use_bvh
    assert L.oracle_ctr_light_batch(C.byref(d), int(bvh), dptr(o), seed, n, dptr(out)) == 0
    return out
