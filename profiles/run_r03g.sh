#!/bin/bash
# r03g: (1) Perlin noise as 8 FMA corner dots + 7 lerps on the device (PL) vs the reference's
# weight-product order (base); (2) persistent 16-wave blocks for the plain flat instance too
# (PF); (3) blocks of 1 / 2 waves for the one-unit-per-wave instances (B1, B2).  Parity with
# the PL and PF libraries, then C2/C4 A/B.
set -o pipefail
O=gpurun_out/r03g
mkdir -p $O
export PYTHONPATH=$PWD/real-time-ray-tracing-engine_amd:$PWD/tests:$PWD
D=$PWD/real-time-ray-tracing-engine_amd
RTX_LIB=$D/build_dbgPL/librtx_hip.so timeout -k 10 400 python -u -m pytest tests/test_gpu_instances.py tests/test_gpu_parity.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/gpu_tests_pl.log 2>&1 || { tail -40 $O/gpu_tests_pl.log; exit 1; }
tail -1 $O/gpu_tests_pl.log
RTX_LIB=$D/build_dbgPF/librtx_hip.so timeout -k 10 400 python -u -m pytest tests/test_gpu_instances.py tests/test_gpu_parity.py tests/test_multi.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/gpu_tests_pf.log 2>&1 || { tail -40 $O/gpu_tests_pf.log; exit 1; }
tail -1 $O/gpu_tests_pf.log
bash profiles/ab.sh $O/ab.log "C4" "base PL B1 B2" 2 || exit 1
bash profiles/ab.sh $O/ab.log "C2" "base PF B1 B2" 2 || exit 1
echo done
