#!/bin/bash
# r03aa: the camera frame read afresh from the kernarg segment at each refill in the plain
# BVH instances too (CF: persistent instance spills 4 -> 0 VGPRs, 24 -> 17 SGPRs): parity, C3 A/B
set -o pipefail
O=gpurun_out/r03aa
mkdir -p $O
export PYTHONPATH=$PWD/real-time-ray-tracing-engine_amd:$PWD/tests:$PWD
RTX_LIB=$PWD/real-time-ray-tracing-engine_amd/build_dbgCF/librtx_hip.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_persistent.py tests/test_c5.py tests/test_bvh4.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
bash profiles/ab.sh $O/ab.log "C3" "base CF" 3 || exit 1
echo done
