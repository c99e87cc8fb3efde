"""The CPU backend's binding (build/librtx_cpu.so, include/rt_cpu.h).

The reference renders on the host when its CLI gets -p without -g
(StaticCamera::render_cpu, StaticCamera.cpp:32-134).  CpuRenderer is that
role behind the same call shapes as rtx.render.Renderer's device calls, so a
caller that chose the CPU (bench.py --device cpu, the launcher tests of its
multi-rank path) drives it like a GPU scene: render_device() writes a host
tensor's memory instead of device memory, in the GPU library's layouts
(RT_LAYOUT_FRAME, RT_LAYOUT_TILES with or without stratum chunks), and
last_kernel_ms() is the host time of the last call.

It is an explicit choice, never a fallback: nothing in rtx/ loads this module
on its own, and librtx_hip.so never loads librtx_cpu.so.
"""
import ctypes as C
import os
import time

from . import abi
from .lib import PKG_DIR, RtError

CPU_LIB_PATH = os.path.join(PKG_DIR, "build", "librtx_cpu.so")
RT_CPU_ABI_VERSION = 2

_lib = None


def load_cpu():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(CPU_LIB_PATH):
        raise RuntimeError("CPU backend %s is not built (run `make -C %s`)" % (CPU_LIB_PATH, PKG_DIR))
    L = C.CDLL(CPU_LIB_PATH)
    P = C.POINTER
    L.rt_cpu_abi_version.restype = C.c_int
    L.rt_cpu_last_error.restype = C.c_char_p
    L.rt_cpu_default_threads.restype = C.c_int
    L.rt_cpu_render.argtypes = [P(abi.SceneDesc), P(abi.Frame), P(abi.RenderParams), C.c_int32,
                                P(C.c_double)]
    L.rt_cpu_render.restype = C.c_int
    if L.rt_cpu_abi_version() != RT_CPU_ABI_VERSION:
        raise RuntimeError("rt_cpu ABI version mismatch: library %d, bindings %d"
                           % (L.rt_cpu_abi_version(), RT_CPU_ABI_VERSION))
    _lib = L
    return L


def default_threads():
    """The CPUs this process may use (affinity mask, cgroup quota)."""
    return int(load_cpu().rt_cpu_default_threads())


class CpuRenderer:
    """A scene rendered by the CPU backend on `threads` host threads (0: the
    library default).  The scene description is compiled per call (the
    backend keeps no state between calls)."""

    def __init__(self, scene, threads=0):
        self.lib = load_cpu()
        self.scene_desc = scene
        self._desc = scene.desc()
        self.threads = int(threads)
        self._ms = 0.0

    def close(self):
        pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def render_device(self, frame, host_ptr, stream_ptr=None, seed=0, rows=(0, 0), samples=(0, -1),
                      output=abi.RT_OUT_SUM, accumulate=0, tiles=(0, 1), layout=abi.RT_LAYOUT_FRAME,
                      chunks=1):
        """rt_render_device's call on the host: overwrite the memory at
        `host_ptr` (a CPU tensor's data_ptr()).  chunks = RT_CHUNKS_AUTO (the
        GPU library's own work units, which return tile sums) returns the tile
        sums here too: the CPU adds a pixel's strata in stratum order, one
        unit per tile.  `stream_ptr` is ignored (the call is synchronous)."""
        from .render import Renderer
        if accumulate:
            raise ValueError("the CPU backend writes its output (accumulate 0)")
        if chunks == abi.RT_CHUNKS_AUTO:
            if layout != abi.RT_LAYOUT_TILES or output != abi.RT_OUT_SUM:
                raise ValueError("RT_CHUNKS_AUTO returns raw tile sums: RT_LAYOUT_TILES, RT_OUT_SUM")
            chunks = 0
        p = Renderer.params(seed, rows, samples, output, 0, tiles, layout, chunks)
        t0 = time.perf_counter()
        rc = self.lib.rt_cpu_render(C.byref(self._desc), C.byref(frame), C.byref(p), self.threads,
                                    C.cast(C.c_void_p(host_ptr), C.POINTER(C.c_double)))
        self._ms = (time.perf_counter() - t0) * 1e3
        if rc != abi.RT_OK:
            msg = self.lib.rt_cpu_last_error()
            raise RtError(rc, msg.decode() if msg else "")

    def last_kernel_ms(self):
        return self._ms
