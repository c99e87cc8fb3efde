#!/bin/bash
# r05x: follow-ups of r05w -- a quarter-slot tail for every frame plan (C2-C4),
# and 8-way subset tails of 125 vs 250 per mille (C2, C3)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05x
mkdir -p $O
bash profiles/ab.sh $O/ab.log "C2 C3 C4" "base RTX_TUNING=tail_tiles=0.25" 3 || exit 1
for c in C2 C3; do
  timeout -k 10 600 python tools/shard_sim.py --config $c --n 8 --plan auto --reps 3 --tuning '{"sub_tail_permille": 250}' '{"sub_tail_permille": 125}' '{"sub_tail_permille": 250}' '{"sub_tail_permille": 125}' > $O/sim_$c.log 2>&1 || { tail $O/sim_$c.log; exit 1; }
done
python - <<'PY'
import json
for c in ("C2", "C3"):
    for l in open("gpurun_out/r05x/sim_%s.log" % c):
        if l.startswith("{"):
            d = json.loads(l)
            print(c, d.get("tuning"), d["tiles_ms"], max(d["tiles_rank_ms"]), d["rank0_path_trip_lane_use"])
PY
