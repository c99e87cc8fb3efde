#!/bin/bash
# r02af: persistent waves only in a dedicated chunked-frame instance whose
# fixed launch fields are constants (base) vs the persistent loop in the plain
# instances (P0): parity + C2/C3/C4 A/B
set -o pipefail
O=gpurun_out/r02af
mkdir -p $O
export PYTHONPATH=$PWD/real-time-ray-tracing-engine_amd:$PWD/tests:$PWD
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_instances.py tests/test_bvh4.py tests/test_multi.py tests/test_device_bvh.py tests/test_bench_contract.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
bash profiles/ab_variants.sh base P0 base P0 > $O/ab.log 2>&1 || exit 1
cat $O/ab.log
