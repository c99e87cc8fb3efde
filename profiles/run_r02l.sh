#!/bin/bash
# r02l: full GPU suite after the 4-wide BVH + RCCL world-of-one exchange tests
set -o pipefail
mkdir -p gpurun_out/r02l
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r02l/gpu_tests.log 2>&1
