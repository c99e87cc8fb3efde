#!/bin/bash
# r06ad: 8-way C2 shares (tools/shard_sim.py --n 8): r06zz read 0.85-0.87 ms per share
# against round 5's 0.80-0.82 -- the pre-probe build (build_dbgR = commit 883e2c5: the
# plain instances re-measure every launch) vs build/ (the probe's order), probe of 64
# strata, plan order
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06ad
mkdir -p $O
B=$PWD/real-time-ray-tracing-engine_amd/build/librtx_hip.so
R=$PWD/real-time-ray-tracing-engine_amd/build_dbgR/librtx_hip.so
sim() { # label lib tuning-json
  RTX_LIB=$2 timeout -k 10 200 python tools/shard_sim.py --config C2 --n 8 --tuning "$3" | python -c "
import json,sys
for l in sys.stdin:
    if l.startswith('{'):
        d=json.loads(l); print('$1', d['N'], d['t1_ms'], max(d['tiles_rank_ms']), d['tiles_rank_ms'], flush=True)"
}
for r in 1 2; do
  sim pre_probe $R null || exit 1
  sim probe16 $B null || exit 1
  sim probe64 $B '{"probe_strata": 64}' || exit 1
  sim plan_order $B '{"no_tile_order": 1}' || exit 1
  sim pre_plan_order $R '{"no_tile_order": 1}' || exit 1
done 2>&1 | tee $O/sim8_C2.log
echo done
