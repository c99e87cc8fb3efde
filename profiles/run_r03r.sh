#!/bin/bash
# r03r: fp32 Perlin octaves (lattice cell and offsets in fp64, corner dots, blend and
# octave sum in fp32; fp32 LDS gradient copy): noise-instance parity, then C4 A/B against
# the fp64 octaves (base)
set -o pipefail
O=gpurun_out/r03r
mkdir -p $O
export PYTHONPATH=$PWD/real-time-ray-tracing-engine_amd:$PWD/tests:$PWD
RTX_LIB=$PWD/real-time-ray-tracing-engine_amd/build_dbgPF/librtx_hip.so timeout -k 10 400 python -u -m pytest tests/test_lds_perlin.py tests/test_gpu_instances.py tests/test_gpu_parity.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
bash profiles/ab.sh $O/ab.log "C4" "PF base" 3 || exit 1
echo done
