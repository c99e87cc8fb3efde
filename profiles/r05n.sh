#!/bin/bash
# r05n: RT_CHUNKS_AUTO (library head/tail units for a tile subset) -- GPU tests,
# then 8-way C2 shares: the chunk plan vs the subset plan over a tuning sweep
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05n
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_subset_auto.py > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 300 python tools/shard_sim.py --config C2 --n 8 --units 32768 > $O/sim_C2.log 2>&1 || { tail $O/sim_C2.log; exit 1; }
T=()
for h in 8 16 32 64; do for pm in -1 250 500 1000; do for sp in 2 4; do
  [ $pm = -1 ] && [ $sp = 4 ] && continue
  T+=("{\"sub_head_strata\": $h, \"sub_tail_permille\": $pm, \"sub_tail_split\": $sp}")
done; done; done
timeout -k 10 600 python tools/shard_sim.py --config C2 --n 8 --plan auto --reps 3 --tuning "${T[@]}" >> $O/sim_C2.log 2>&1 || { tail $O/sim_C2.log; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/r05n/sim_C2.log"):
    if l.startswith("{"):
        d = json.loads(l)
        print(d["plan"], d.get("tuning"), d["tiles_ms"], d["speedup_k"], d["rank0_path_trip_lane_use"], max(d["tiles_rank_ms"]))
PY
