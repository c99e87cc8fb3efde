#!/bin/bash
# r02ag: a persistent chunked-frame instance for the flat sphere world too
# (PF, RT_PERSIST_FLAT=1) vs base (flat keeps one unit per wave): C2 parity + A/B
set -o pipefail
O=gpurun_out/r02ag
mkdir -p $O
export PYTHONPATH=$PWD/real-time-ray-tracing-engine_amd:$PWD/tests:$PWD
RTX_LIB=$PWD/real-time-ray-tracing-engine_amd/build_dbgPF/librtx_hip.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -u -m pytest tests/test_persistent.py -x -v -m gpu --timeout 200 --timeout-method thread > $O/persistent_tests.log 2>&1 || { tail -30 $O/persistent_tests.log; exit 1; }
tail -5 $O/persistent_tests.log
for r in 1 2 3; do
  for v in base PF; do
    if [ $v = base ]; then L=$PWD/real-time-ray-tracing-engine_amd/build/librtx_hip.so; else L=$PWD/real-time-ray-tracing-engine_amd/build_dbg$v/librtx_hip.so; fi
    RTX_LIB=$L timeout -k 10 200 python bench.py --config C2 --steps 10 --warmup 2 --no-cpu-baseline --pmc off --no-other-configs 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$v', 'C2', d['value'])" || exit 1
  done
done | tee $O/ab.log
