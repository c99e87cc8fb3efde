#!/bin/bash
# r02m: branchless binary node visit (base) vs the branchy form (B0):
# GPU parity of the base build, then C2/C3/C4 and 100k-sphere A/B, interleaved.
set -o pipefail
O=gpurun_out/r02m
mkdir -p $O
export PYTHONPATH=$PWD/real-time-ray-tracing-engine_amd
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_instances.py tests/test_bvh4.py tests/test_device_bvh.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
bash profiles/ab_variants.sh base B0 base B0 > $O/ab.log 2>&1 &&
for v in base B0 base B0; do
  L=$PWD/real-time-ray-tracing-engine_amd/build/librtx_hip.so; [ $v = base ] || L=$PWD/real-time-ray-tracing-engine_amd/build_dbg$v/librtx_hip.so
  echo "== $v" && RTX_LIB=$L timeout -k 10 200 python -u tools/arity_ab.py --no-c3 --n 100000 --rounds 2 || exit 1
done >> $O/ab.log 2>&1
