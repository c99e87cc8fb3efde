#!/bin/bash
# r06ae: subset (tile-shard) launches probed with their own plan at every stratum
# (build_dbgS = -DRT_PLAN_PROBE_EXPERIMENT) vs the 16-strata whole-tile probe (build/)
# and the pre-probe build (build_dbgR, re-measured every launch): 4- and 8-way C2 / C3
# shares on one GPU (tools/shard_sim.py)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06ae
mkdir -p $O
B=$PWD/real-time-ray-tracing-engine_amd/build/librtx_hip.so
R=$PWD/real-time-ray-tracing-engine_amd/build_dbgR/librtx_hip.so
S=$PWD/real-time-ray-tracing-engine_amd/build_dbgS/librtx_hip.so
sim() { # label lib config
  RTX_LIB=$2 timeout -k 10 300 python tools/shard_sim.py --config $3 --n 4 8 | python -c "
import json,sys
for l in sys.stdin:
    if l.startswith('{'):
        d=json.loads(l); print('$1', '$3', d['N'], d['t1_ms'], max(d['tiles_rank_ms']), d['tiles_rank_ms'], flush=True)"
}
for r in 1 2; do
  for c in C2 C3; do
    sim pre_probe $R $c || exit 1
    sim probe16 $B $c || exit 1
    sim plan_probe $S $c || exit 1
  done
done 2>&1 | grep -v amdgpu.ids | tee $O/sim_C2_C3.log
echo done
