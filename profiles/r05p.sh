#!/bin/bash
# r05p: the library subset plan as the tile-shard default -- GPU tests of the
# touched paths, then 1/2/4/8-way shares (C2, C3) and the 8-way C4 / C5 shares,
# chunk plan vs the library plan
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05p
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_subset_auto.py tests/test_dist.py tests/test_bench_contract.py tests/test_multi.py > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
for c in C2 C3; do
  timeout -k 10 300 python tools/shard_sim.py --config $c --n 1 2 4 8 > $O/sim_$c.log 2>&1 || { tail $O/sim_$c.log; exit 1; }
  timeout -k 10 300 python tools/shard_sim.py --config $c --n 1 2 4 8 --plan auto >> $O/sim_$c.log 2>&1 || { tail $O/sim_$c.log; exit 1; }
done
for c in C4 C5; do
  timeout -k 10 400 python tools/shard_sim.py --config $c --n 8 --reps 2 > $O/sim_$c.log 2>&1 || { tail $O/sim_$c.log; exit 1; }
  timeout -k 10 400 python tools/shard_sim.py --config $c --n 8 --reps 2 --plan auto >> $O/sim_$c.log 2>&1 || { tail $O/sim_$c.log; exit 1; }
done
python - <<'PY'
import json
for c in ("C2", "C3", "C4", "C5"):
    for l in open("gpurun_out/r05p/sim_%s.log" % c):
        if l.startswith("{"):
            d = json.loads(l)
            print(c, d["N"], d["plan"], d["tiles_chunks"], d["tiles_ms"], d["speedup_k"], d["rank0_path_trip_lane_use"], max(d["tiles_rank_ms"]))
PY
