#!/bin/bash
# r02ab: persistent waves pulling (tile, stratum chunk) work units from an
# agent-scope counter (default) vs one unit per wave (RT_PERSISTENT=0):
# parity suite, C2/C3/C4 A/B interleaved
set -o pipefail
O=gpurun_out/r02ab
mkdir -p $O
export PYTHONPATH=$PWD/real-time-ray-tracing-engine_amd:$PWD/tests:$PWD
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_instances.py tests/test_bvh4.py tests/test_multi.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for r in 1 2; do
  for v in 1 0; do
    for c in C2 C3 C4; do
      s=3; [ $c = C4 ] && s=1
      RT_PERSISTENT=$v timeout -k 10 200 python bench.py --config $c --steps $s --warmup 1 --no-cpu-baseline --pmc off --no-other-configs 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('persistent=$v', '$c', d['value'])" || exit 1
    done
  done
done | tee $O/ab.log
