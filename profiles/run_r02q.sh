#!/bin/bash
# r02q: packed fp32 slab tests in the 4-wide walk (base) vs per-child (K0)
set -o pipefail
O=gpurun_out/r02q
mkdir -p $O
export PYTHONPATH=$PWD/real-time-ray-tracing-engine_amd
timeout -k 10 300 python -u -m pytest tests/test_bvh4.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
B=$PWD/real-time-ray-tracing-engine_amd/build/librtx_hip.so
K=$PWD/real-time-ray-tracing-engine_amd/build_dbgK0/librtx_hip.so
for L in $B $K $B $K; do
  echo "== $L" && RTX_LIB=$L timeout -k 10 300 python -u tools/arity_ab.py --n 100000 1000000 --rounds 2 || exit 1
done > $O/ab.log 2>&1
