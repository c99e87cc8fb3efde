#!/bin/bash
# r02p: sphere roots of transformed items through a by-value reciprocal (base)
# vs the pointer-to-local form (P, previous commit): parity + cornell/C3 A/B
set -o pipefail
O=gpurun_out/r02p
mkdir -p $O
export PYTHONPATH=$PWD/real-time-ray-tracing-engine_amd
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_instances.py tests/test_bvh4.py tests/test_edge_cases.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
B=$PWD/real-time-ray-tracing-engine_amd/build/librtx_hip.so
P=$PWD/real-time-ray-tracing-engine_amd/build_dbgP/librtx_hip.so
for L in $B $P $B $P; do
  RTX_LIB=$L timeout -k 10 200 python -u tools/scene_rate.py --scenes cornell cornell_fog --spp 64 || exit 1
done > $O/ab.log 2>&1
