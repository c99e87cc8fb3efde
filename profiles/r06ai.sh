#!/bin/bash
# r06ai: first-measure order for the plain BVH worlds' tile subsets too (build_dbgX =
# -DRT_COST_BVH_EXPERIMENT: COST variants of the plain BVH instances, persistent ones
# included) vs the probe's order (build/) -- 4- and 8-way C3 shares, settle 1 and 4
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06ai
mkdir -p $O
B=$PWD/real-time-ray-tracing-engine_amd/build/librtx_hip.so
X=$PWD/real-time-ray-tracing-engine_amd/build_dbgX/librtx_hip.so
sim() { # label lib settle
  RTX_LIB=$2 timeout -k 10 300 python tools/shard_sim.py --config C3 --n 4 8 --settle $3 | python -c "
import json,sys
for l in sys.stdin:
    if l.startswith('{'):
        d=json.loads(l); print('$1', 'settle', $3, d['N'], d['t1_ms'], max(d['tiles_rank_ms']), d['speedup_k'], flush=True)"
}
for r in 1 2; do
  for k in 1 3; do
    sim probe $B $k || exit 1
    sim first_measure $X $k || exit 1
  done
done 2>&1 | grep -v amdgpu.ids | tee $O/sim_C3.log
echo done
