#!/bin/bash
# r06ag: 8-way C2 shares after 1 and 4 untimed launches of the same share (shard_sim
# --settle): pre-probe build (build_dbgR), COST subsets re-measuring every launch after
# the probe (build/), first launch of a subset shape measuring its own costs in plan
# order and the later ones taking that order in the plain instance (build_dbgV)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06ag
mkdir -p $O
B=$PWD/real-time-ray-tracing-engine_amd/build/librtx_hip.so
R=$PWD/real-time-ray-tracing-engine_amd/build_dbgR/librtx_hip.so
V=$PWD/real-time-ray-tracing-engine_amd/build_dbgV/librtx_hip.so
sim() { # label lib settle
  RTX_LIB=$2 timeout -k 10 300 python tools/shard_sim.py --config C2 --n 8 --settle $3 | python -c "
import json,sys
for l in sys.stdin:
    if l.startswith('{'):
        d=json.loads(l); print('$1', 'settle', $3, d['N'], d['t1_ms'], max(d['tiles_rank_ms']), d['tiles_rank_ms'], flush=True)"
}
for r in 1 2; do
  for k in 1 4; do
    sim pre_probe $R $k || exit 1
    sim cost_remeasure $B $k || exit 1
    sim first_measure $V $k || exit 1
  done
done 2>&1 | grep -v amdgpu.ids | tee $O/sim8_C2.log
echo done
