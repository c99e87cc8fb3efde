#!/bin/bash
# r03w: at-use sincos constants in the plain BVH instances only (product), vs the hoisted form
# everywhere (K0, the r03t product) on C2/C3/C4; the packed binary node visit on top (PK) on C3
# (the persistent instance now spills 4 VGPRs with either visit)
set -o pipefail
O=gpurun_out/r03w
mkdir -p $O
export PYTHONPATH=$PWD/real-time-ray-tracing-engine_amd:$PWD/tests:$PWD
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
RTX_LIB=$PWD/real-time-ray-tracing-engine_amd/build_dbgPK/librtx_hip.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_persistent.py tests/test_bvh4.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/gpu_tests_pk.log 2>&1 || { tail -40 $O/gpu_tests_pk.log; exit 1; }
tail -1 $O/gpu_tests_pk.log
bash profiles/ab.sh $O/ab.log "C3" "base K0 PK" 3 || exit 1
bash profiles/ab.sh $O/ab.log "C2 C4" "base K0" 2 || exit 1
echo done
