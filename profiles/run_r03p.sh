#!/bin/bash
# r03p: merged regeneration in the flat instance (refills inside the trip, sharing the
# shading event's Philox block): flat-instance parity, then C2 A/B against the old
# trip (M0) and merged refill thresholds 8 / 16 (M8, M16; base: 1)
set -o pipefail
O=gpurun_out/r03p
mkdir -p $O
export PYTHONPATH=$PWD/real-time-ray-tracing-engine_amd:$PWD/tests:$PWD
timeout -k 10 400 python -u -m pytest tests/test_gpu_instances.py tests/test_gpu_parity.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
bash profiles/ab.sh $O/ab.log "C2" "base M0 M8 M16" 3 || exit 1
echo done
