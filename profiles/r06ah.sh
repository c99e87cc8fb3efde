#!/bin/bash
# r06ah: first-measure subsets productized (build/): tile-order / multi / dist / subset
# GPU tests, 2/4/8-way C2 shares (settle 1 and 4); full C2 frames ordered the same way
# (build_dbgW: the first frame launch measures in the COST instance) vs the probe (build/)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06ah
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_tile_order.py tests/test_multi.py tests/test_dist.py tests/test_subset_auto.py tests/test_launcher.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
B=$PWD/real-time-ray-tracing-engine_amd/build/librtx_hip.so
W=$PWD/real-time-ray-tracing-engine_amd/build_dbgW/librtx_hip.so
for k in 1 4; do
  timeout -k 10 300 python tools/shard_sim.py --config C2 --n 2 4 8 --settle $k | python -c "
import json,sys
for l in sys.stdin:
    if l.startswith('{'):
        d=json.loads(l); print('first_measure settle', $k, d['N'], d['t1_ms'], max(d['tiles_rank_ms']), d['speedup_k'], flush=True)" || exit 1
done 2>&1 | grep -v amdgpu.ids | tee $O/sim_C2.log
for r in 1 2 3; do
  for v in B W; do
    L=$B; [ $v = W ] && L=$W
    RTX_LIB=$L timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --pmc off --no-other-configs 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$v', 'C2', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], flush=True)" || exit 1
  done
done 2>&1 | tee $O/ab_C2_frames.log
echo done
