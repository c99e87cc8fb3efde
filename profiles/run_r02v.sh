#!/bin/bash
# r02v: time-linear BVH boxes (RT_FEAT_MOTION): GPU parity, then C3 A/B
set -o pipefail
O=gpurun_out/r02v
mkdir -p $O
export PYTHONPATH=$PWD/real-time-ray-tracing-engine_amd:$PWD/tests:$PWD
timeout -k 10 500 python -u -m pytest tests/test_motion.py tests/test_gpu_parity.py tests/test_gpu_instances.py tests/test_bvh4.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -u tools/motion_ab.py --rounds 3 > $O/ab.log 2>&1
