"""rtx — MI355X-native path-tracing hot path (Python host side).

The per-pixel work runs in hand-written HIP kernels for gfx950 behind the C ABI
of include/rt_api.h (build/librtx_hip.so).  This package parses JSON scenes,
mirrors the reference's StaticCamera flow and writes PPM files.
"""
from . import abi  # noqa: F401
from .scene import load_scene, SceneDescription, SceneError  # noqa: F401
from .ppm import to_bytes, ppm_bytes, write_ppm  # noqa: F401
