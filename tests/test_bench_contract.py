"""bench.py's output contract, run end to end on one GPU at the C1 size.

One bench process per case (sequential, one GPU user at a time): the JSON line
carries the driver's keys, the roofline / cpu-baseline-free fields, and its
--check compares the timed frame with a single-device render (both N=1 layouts:
frame-direct and tile work units + reorder)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

KEYS = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
        "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config", "roofline")


def _bench(*extra):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--config", "C1", "--steps", "2",
           "--warmup", "1", "--no-cpu-baseline", "--check", *extra]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-2000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.mark.gpu
@pytest.mark.parametrize("layout", ["frame", "tiles"])
def test_bench_line(layout):
    d = _bench("--n1-layout", layout)
    for k in KEYS:
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 2 and d["dtype"] == "f64"
    assert d["value"] > 0 and d["unit"] == "Msamples/s"
    rf = d["roofline"]
    assert rf["kernel_ms"] > 0 and rf["achieved"] > 0 and rf["frac"] == pytest.approx(
        rf["achieved"] / rf["peak"], rel=1e-3)
    assert d["config"]["width"] == 400 and d["config"]["spp"] == 9
    assert d["check"]["ok"], d["check"]
