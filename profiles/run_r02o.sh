#!/bin/bash
# r02o: boundary candidate flags packed into an integer (no scratch byte array):
# parity, then C4 bench with live PMC passes (scratch write traffic), C2/C3 lines
set -o pipefail
O=gpurun_out/r02o
mkdir -p $O
export PYTHONPATH=$PWD/real-time-ray-tracing-engine_amd
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_instances.py tests/test_bvh4.py tests/test_statistical_parity.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 600 python bench.py --config C4 --steps 2 --warmup 1 --no-cpu-baseline --no-other-configs > $O/bench_C4.json 2> $O/bench_C4.err
