#!/bin/bash
# r03u: the persistent BVH instance at 3 waves/SIMD (12-wave blocks, one per CU, 152 VGPRs,
# no spills; W3) and with the packed binary node visit (W3PK) vs the product (16-wave blocks
# at 4 waves/SIMD, 20 spilled VGPRs): W3PK parity on the persistent and BVH tests, C3 A/B
set -o pipefail
O=gpurun_out/r03u
mkdir -p $O
export PYTHONPATH=$PWD/real-time-ray-tracing-engine_amd:$PWD/tests:$PWD
RTX_LIB=$PWD/real-time-ray-tracing-engine_amd/build_dbgW3PK/librtx_hip.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_c5.py tests/test_bvh4.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
bash profiles/ab.sh $O/ab.log "C3" "base W3 W3PK" 3 || exit 1
echo done
