#!/bin/bash
# r02ao: the persistent instance reads its per-unit launch fields afresh from
# the kernarg segment (base, RT_KARG_FRESH=1: SGPR spills 72 -> 22, VGPR 21 -> 17)
# vs held across the unit (K0): persistence + parity tests, C3 A/B
set -o pipefail
O=gpurun_out/r02ao
mkdir -p $O
export PYTHONPATH=$PWD/real-time-ray-tracing-engine_amd:$PWD/tests:$PWD
timeout -k 10 300 python -u -m pytest tests/test_persistent.py tests/test_gpu_parity.py tests/test_bench_contract.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for r in 1 2 3; do
  for v in base K0; do
    if [ $v = base ]; then L=$PWD/real-time-ray-tracing-engine_amd/build/librtx_hip.so; else L=$PWD/real-time-ray-tracing-engine_amd/build_dbg$v/librtx_hip.so; fi
    RTX_LIB=$L timeout -k 10 200 python bench.py --config C3 --steps 3 --warmup 1 --no-cpu-baseline --pmc off --no-other-configs 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$v', 'C3', d['value'])" || exit 1
  done
done | tee $O/ab.log
