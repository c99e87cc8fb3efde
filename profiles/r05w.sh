#!/bin/bash
# r05w: C2's frame plan re-swept with cost-ordered dispatch on (tail tiles per
# slot, tail split, head strata), and the 8-way subset plan
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05w
mkdir -p $O
bash profiles/ab.sh $O/ab.log "C2" "base RTX_TUNING=tail_tiles=0.25 RTX_TUNING=tail_tiles=1.0 RTX_TUNING=tail_split=4 RTX_TUNING=tail_split=16 RTX_TUNING=tail_tiles=1.0,tail_split=4 RTX_TUNING=head_strata=32 RTX_TUNING=tail_tiles=0.25,tail_split=16" 2 || exit 1
T=()
for h in 12 16 24; do for pm in 125 250 500; do
  T+=("{\"sub_head_strata\": $h, \"sub_tail_permille\": $pm, \"sub_tail_split\": 2}")
done; done
timeout -k 10 600 python tools/shard_sim.py --config C2 --n 8 --plan auto --reps 3 --tuning "${T[@]}" > $O/sim_C2.log 2>&1 || { tail $O/sim_C2.log; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/r05w/sim_C2.log"):
    if l.startswith("{"):
        d = json.loads(l)
        print(d.get("tuning"), d["tiles_ms"], max(d["tiles_rank_ms"]), d["rank0_path_trip_lane_use"])
PY
