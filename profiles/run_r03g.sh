#!/bin/bash
# r03g: Perlin noise as 8 FMA corner dots + 7 lerps on the device (PL) vs the reference's
# weight-product order (base): parity of every instance with the PL library, C4 A/B
set -o pipefail
O=gpurun_out/r03g
mkdir -p $O
export PYTHONPATH=$PWD/real-time-ray-tracing-engine_amd:$PWD/tests:$PWD
RTX_LIB=$PWD/real-time-ray-tracing-engine_amd/build_dbgPL/librtx_hip.so timeout -k 10 400 python -u -m pytest tests/test_gpu_instances.py tests/test_gpu_parity.py tests/test_statistical_parity.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
bash profiles/ab.sh $O/ab.log "C4" "base PL" 3 || exit 1
echo done
