#!/bin/bash
# r02k: 4-wide BVH -- GPU parity tests, then binary vs 4-wide A/B (C3, 20k/100k/1M spheres)
set -o pipefail
mkdir -p gpurun_out/r02k
export PYTHONPATH=$PWD/real-time-ray-tracing-engine_amd:$PWD/tests:$PWD
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_bvh4.py tests/test_device_bvh.py tests/test_gpu_instances.py > gpurun_out/r02k/tests.log 2>&1 &&
timeout -k 10 400 python -u tools/arity_ab.py --n 20000 100000 1000000 --rounds 3 > gpurun_out/r02k/ab.log 2>&1
