"""pytest configuration: `gpu` marker + import paths.

CPU suite:  python -m pytest tests -q -m "not gpu"
GPU suite:  python -m pytest tests -q -m gpu       (real MI355X, via the C ABI)
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "real-time-ray-tracing-engine_amd")
for p in (PKG, os.path.join(ROOT, "tests"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); runs through the C ABI")
