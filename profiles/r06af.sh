#!/bin/bash
# r06af: tile-subset launches of the flat world measuring their own costs again (the
# COST instance, build/) vs the pre-probe build (build_dbgR) -- 2/4/8-way C2 shares on
# one GPU; the tile-order / multi / dist GPU tests; C2 default-line check
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06af
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_tile_order.py tests/test_multi.py tests/test_dist.py tests/test_subset_auto.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
B=$PWD/real-time-ray-tracing-engine_amd/build/librtx_hip.so
R=$PWD/real-time-ray-tracing-engine_amd/build_dbgR/librtx_hip.so
sim() { # label lib config
  RTX_LIB=$2 timeout -k 10 300 python tools/shard_sim.py --config $3 --n 2 4 8 | python -c "
import json,sys
for l in sys.stdin:
    if l.startswith('{'):
        d=json.loads(l); print('$1', '$3', d['N'], d['t1_ms'], max(d['tiles_rank_ms']), d['tiles_rank_ms'], flush=True)"
}
for r in 1 2; do
  sim pre_probe $R C2 || exit 1
  sim cost_subsets $B C2 || exit 1
done 2>&1 | grep -v amdgpu.ids | tee $O/sim_C2.log
for r in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --pmc off --no-other-configs 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('C2', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], flush=True)" || exit 1
done 2>&1 | tee $O/c2.log
echo done
