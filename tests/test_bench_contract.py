"""bench.py's output contract, run end to end on one GPU at the C1 size (N=1 and
a 2-rank rehearsal of the N>1 path).

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


def _bench(*extra, timeout=110):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--config", "C1", "--steps", "2",
           "--warmup", "1", "--no-cpu-baseline", "--no-other-configs", "--check", *extra]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-2000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.mark.gpu
@pytest.mark.parametrize("layout", ["frame", "tiles"])
def test_bench_line(layout):
    d = _bench("--n1-layout", layout, "--pmc", "file")
    for k in KEYS:
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 2 and d["dtype"] == "f64"
    assert d["value"] > 0 and d["unit"] == "Msamples/s"
    rf = d["roofline"]
    assert rf["bound"] == "valu" and rf["unit"] == "TFLOP/s" and rf["kernel_ms"] > 0
    assert rf["peak"] == 78.6 and 0 < rf["frac"] <= 1
    assert rf["frac"] == pytest.approx(rf["achieved"] / rf["peak"], rel=1e-3)
    assert 0 < rf["valu_busy"] <= 1 and 0 < rf["f64_inst_share"] <= 1
    assert "committed" in rf["pmc_source"]
    assert d["config"]["width"] == 400 and d["config"]["spp"] == 9
    assert d["check"]["ok"], d["check"]


@pytest.mark.gpu
def test_bench_line_live_pmc():
    """Default --pmc auto: bench.py runs the rocprofv3 PMC passes (VALU, FETCH_SIZE,
    WRITE_SIZE) on this build before its timed run; the roofline is the fp64
    FLOP rate against the fp64 vector peak (<= 1), VALU-busy beside it, and
    traffic the PMC HBM bytes."""
    d = _bench(timeout=400)
    rf = d["roofline"]
    assert rf["pmc_source"].startswith("live"), rf.get("pmc_source")
    assert 0 < rf["frac"] <= 1 and rf["traffic"] > 0 and 0 < rf["valu_busy"] <= 1
    assert rf["hbm_frac"] < 1


@pytest.mark.gpu
@pytest.mark.parametrize("config", ["C2", "C3"])
def test_bench_roofline_counts_issue_and_lanes(config):
    """The live PMC figures at the headline (C2) and the BVH (C3) configs
    (VERDICT r3 item 3): valu_busy -- quad-cycles in which the VALU issues at
    all, (SQ_ACTIVE_INST_VALU - SQ_ACTIVE_INST_VALU2) over the SIMD quad-cycles
    -- is <= 1 while rocprofv3's VALUBusy (valu_issue_ratio) may exceed it
    under gfx950's dual issue; the lane-weighted fp64 fraction (the issued
    rate x SQ_THREAD_CYCLES_VALU / 64 SQ_ACTIVE_INST_VALU) sits beside frac,
    below it."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--config", config, "--steps", "2",
           "--warmup", "1", "--no-cpu-baseline", "--no-other-configs"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-2000:]
    rf = json.loads(r.stdout.strip().splitlines()[-1])["roofline"]
    assert rf["pmc_source"].startswith("live"), rf.get("pmc_source")
    assert 0 < rf["valu_busy"] <= 1, rf["valu_busy"]
    assert rf["valu_issue_ratio"] >= rf["valu_busy"]
    assert 0 < rf["valu_lane_fraction"] <= 1
    assert 0 < rf["frac_active_lanes"] <= rf["frac"] <= 1
    assert rf["frac_active_lanes"] == pytest.approx(rf["frac"] * rf["valu_lane_fraction"], rel=2e-3)


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.gpu
@pytest.mark.parametrize("shard", ["tiles", "strata"])
def test_bench_two_ranks_one_gpu(shard):
    """The N>1 bench path (tile gather / stratum reduce, double-buffered) with 2
    ranks sharing cuda:0 and gloo standing in for RCCL; rank 0's frame must match
    a single-device render (--check)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--config", "C1", "--steps", "2",
           "--warmup", "1", "--backend", "gloo", "--share-device", "--check", "--shard", shard]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=110,
                       env=dict(os.environ, MASTER_ADDR="127.0.0.1"))
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["n_gpus"] == 2 and d["value"] > 0
    assert d["check"]["ok"], d["check"]
    # per-rank diagnostics: kernel ms of each rank, rank 0's exchange wait
    rk = d["ranks"]
    assert len(rk["per_rank_kernel_ms"]) == 2 and len(rk["per_rank_exchange_ms"]) == 2
    assert 0 < rk["kernel_ms_min"] <= rk["kernel_ms_mean"] <= rk["kernel_ms_max"]
    assert rk["exchange_ms_rank0"] >= 0 and rk["exchange_ms_max"] >= rk["exchange_ms_rank0"]


@pytest.mark.gpu
@pytest.mark.parametrize("shard", ["tiles", "strata"])
def test_bench_rccl_exchange_world_of_one(shard):
    """The RCCL calls of the N>1 path (async gather of tile sums / async reduce of
    stratum sums, .wait() before reuse of the double buffer) on a real
    process group over RCCL -- a world of one, the most this one-GPU box can run
    (RCCL refuses two ranks on one device); the frame must match a
    single-device render (--check)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "1", "--config", "C1", "--steps", "3",
           "--warmup", "1", "--backend", "nccl", "--pg-rehearsal", "--check", "--shard", shard,
           "--pmc", "off", "--no-cpu-baseline", "--no-other-configs"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=110,
                       env=dict(os.environ, MASTER_ADDR="127.0.0.1"))
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["n_gpus"] == 1 and d["value"] > 0
    assert "RCCL" in d["config"]["parallelism"], d["config"]
    assert d["check"]["ok"], d["check"]
