#!/bin/bash
# r02r: camera-ray constants from an LDS copy in the rich instances (base) vs
# kernel-argument SGPRs (L0): parity + C4/cornell/cornell_fog-variants A/B
set -o pipefail
O=gpurun_out/r02r
mkdir -p $O
export PYTHONPATH=$PWD/real-time-ray-tracing-engine_amd
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_instances.py tests/test_bvh4.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
B=$PWD/real-time-ray-tracing-engine_amd/build/librtx_hip.so
L=$PWD/real-time-ray-tracing-engine_amd/build_dbgL0/librtx_hip.so
for X in $B $L $B $L; do
  RTX_LIB=$X timeout -k 10 200 python -u tools/scene_rate.py --scenes cornell_fog cornell --spp 256 || exit 1
done > $O/ab.log 2>&1
