#!/bin/bash
# r05o: 8-way shares of C2 / C3 / C4 under the RT_CHUNKS_AUTO subset plan
# (sweep of head strata, tail share and split) against the chunk plan
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05o
mkdir -p $O
run() { # config, head strata list
  local c=$1; shift
  timeout -k 10 300 python tools/shard_sim.py --config $c --n 8 > $O/sim_$c.log 2>&1 || { tail $O/sim_$c.log; return 1; }
  local T=()
  for h in "$@"; do for pm in 250 500; do for sp in 2 4; do
    T+=("{\"sub_head_strata\": $h, \"sub_tail_permille\": $pm, \"sub_tail_split\": $sp}")
  done; done; done
  timeout -k 10 900 python tools/shard_sim.py --config $c --n 8 --plan auto --reps 3 --tuning "${T[@]}" >> $O/sim_$c.log 2>&1 || { tail $O/sim_$c.log; return 1; }
}
run C2 12 16 20 && run C3 16 32 64 128 && run C4 32 64 128 256 || exit 1
python - <<'PY'
import json
for c in ("C2", "C3", "C4"):
    for l in open("gpurun_out/r05o/sim_%s.log" % c):
        if l.startswith("{"):
            d = json.loads(l)
            print(c, d["plan"], d.get("tuning"), d["tiles_ms"], d["speedup_k"], d["rank0_path_trip_lane_use"], max(d["tiles_rank_ms"]))
PY
