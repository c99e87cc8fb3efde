"""bench.py as its own launcher: `bench.py --gpus N` with
no WORLD_SIZE in the environment starts N rank processes itself (torchrun's
variables, 127.0.0.1 rendezvous), relays rank 0's JSON line and fails when
any rank fails; with a launcher, the world it was given must be --gpus.

These run on the CPU: --device cpu puts every rank on the CPU backend
(librtx_cpu.so, the GPU kernel's per-path source compiled for the host) with
the gloo exchange, so the launcher, the process group, the tile gather /
stratum reduce and the frame check are the ones an 8-GPU run takes -- only
the render backend differs.  The reference renders on one device
(StaticCamera.cpp:235-300); the multi-rank path is this framework's."""
import json
import os
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT", "LOCAL_WORLD_SIZE")}
    env.update(kw)
    return env


def _run(args, timeout=240, **env):
    return subprocess.run([sys.executable, BENCH] + args, cwd=ROOT, capture_output=True, text=True,
                          timeout=timeout, env=_env(**env))


def _line(r):
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.strip().splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout  # one JSON line: rank 0's, relayed
    return json.loads(lines[0])


@pytest.mark.parametrize("shard", ["tiles", "strata"])
def test_bench_launches_its_own_ranks(shard):
    """--gpus 2 without torchrun: two ranks, both reached by the exchange
    (ranks_seen from an all_gather of rank ids), and rank 0's frame equals a
    one-rank render of all strata (--check)."""
    r = _run(["--gpus", "2", "--backend", "gloo", "--share-device", "--config", "C1", "--check",
              "--device", "cpu", "--steps", "2", "--warmup", "1", "--shard", shard])
    d = _line(r)
    assert d["n_gpus"] == 2 and d["ranks_seen"] == 2, d
    assert d["check"]["ok"], d["check"]
    assert d["config"]["launcher"] == "bench.py" and "x2" in d["config"]["parallelism"]
    assert d["value"] > 0 and len(d["ranks"]["per_rank_kernel_ms"]) == 2
    assert "launched 2 ranks" in r.stderr


def test_bench_three_ranks_ragged_tiles():
    """An odd world: 3 ranks over C1's 1,450 tiles (not a multiple of 3)."""
    d = _line(_run(["--gpus", "3", "--backend", "gloo", "--config", "C1", "--check",
                    "--device", "cpu", "--steps", "1", "--warmup", "0", "--spp", "4"]))
    assert d["n_gpus"] == 3 and d["ranks_seen"] == 3 and d["check"]["ok"], d


def test_bench_refuses_more_gpus_than_visible():
    """--gpus N on a box with fewer devices exits non-zero with a message
    before any rank starts (not a 1-rank line that looks like an N-GPU one)."""
    import torch
    n = max(2, torch.cuda.device_count() + 1)
    t0 = time.time()
    r = _run(["--gpus", str(n), "--config", "C1", "--steps", "1", "--warmup", "0"], timeout=120)
    assert r.returncode != 0
    assert "needs %d GPUs" % n in r.stderr and "launched" not in r.stderr
    assert r.stdout.strip() == ""
    assert time.time() - t0 < 100


def test_bench_refuses_a_launcher_world_that_is_not_gpus():
    """Under a launcher (WORLD_SIZE set) the world must be --gpus."""
    r = _run(["--gpus", "3", "--config", "C1", "--device", "cpu", "--backend", "gloo"], timeout=120,
             WORLD_SIZE="2", RANK="0", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT="1")
    assert r.returncode == 2 and "WORLD_SIZE 2" in r.stderr


def test_bench_launcher_fails_when_a_rank_fails():
    """A rank that dies makes the launcher stop the others (which would wait in
    the exchange for ever) and exit non-zero, with no JSON line."""
    t0 = time.time()
    r = _run(["--gpus", "2", "--backend", "gloo", "--share-device", "--config", "C1", "--device",
              "cpu", "--steps", "50", "--warmup", "1", "--fail-rank", "1"], timeout=180)
    assert r.returncode != 0
    assert "rank 1 exited with 3" in r.stderr
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert time.time() - t0 < 150


def test_cpu_device_needs_gloo():
    r = _run(["--gpus", "2", "--device", "cpu", "--backend", "nccl", "--config", "C1"], timeout=60)
    assert r.returncode == 2 and "gloo" in r.stderr


@pytest.mark.gpu
def test_bench_launches_its_own_ranks_on_the_gpu():
    """The same on the GPU box: --gpus 2 without torchrun, both ranks on cuda:0
    (--share-device) with gloo standing in for RCCL (which refuses two ranks on
    one device); the GPU library renders, rank 0's frame matches one device."""
    d = _line(_run(["--gpus", "2", "--backend", "gloo", "--share-device", "--config", "C1",
                    "--check", "--steps", "2", "--warmup", "1"], timeout=200))
    assert d["n_gpus"] == 2 and d["ranks_seen"] == 2 and d["check"]["ok"], d
    assert d["config"]["device"] == "gpu" and d["config"]["launcher"] == "bench.py"
