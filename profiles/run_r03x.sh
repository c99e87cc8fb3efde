#!/bin/bash
# r03x: sincos constants materialised in VGPRs at their use in the rich instances (KV: two
# v_mov_b32 per constant, 20 VGPRs no longer held; 164 VGPRs, no spills), and the same at
# 4 waves/SIMD (KV4: 33 spilled VGPRs): KV parity, C4 A/B
set -o pipefail
O=gpurun_out/r03x
mkdir -p $O
export PYTHONPATH=$PWD/real-time-ray-tracing-engine_amd:$PWD/tests:$PWD
RTX_LIB=$PWD/real-time-ray-tracing-engine_amd/build_dbgKV/librtx_hip.so timeout -k 10 400 python -u -m pytest tests/test_lds_perlin.py tests/test_gpu_instances.py tests/test_gpu_parity.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
bash profiles/ab.sh $O/ab.log "C4" "base KV KV4" 2 || exit 1
echo done
