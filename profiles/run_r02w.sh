#!/bin/bash
# r02w: merged shading (shared unit vector / sincos / first root across the
# material branches) = base vs per-material code (M0): parity + C2/C3/C4 A/B + cornell
set -o pipefail
O=gpurun_out/r02w
mkdir -p $O
export PYTHONPATH=$PWD/real-time-ray-tracing-engine_amd:$PWD/tests:$PWD
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_instances.py tests/test_bvh4.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
bash profiles/ab_variants.sh base M0 base M0 > $O/ab.log 2>&1
