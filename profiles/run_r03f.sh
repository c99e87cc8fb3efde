#!/bin/bash
# r03f: head/tail frame plan (whole tiles or <= 4 head chunks of <= 64 strata, the last
# slots x RTX_TAIL_TILES tiles 8x finer) -- multi/persistent/parity tests, then A/B:
# C2 tail 0.5 (default) vs 0.25 / 1 / uniform; C3 head 4 chunks + tail 0.5 (default) vs
# uniform (RTX_TAIL_TILES=0) / tail 1 / tail 2.
set -o pipefail
O=gpurun_out/r03f
mkdir -p $O
export PYTHONPATH=$PWD/real-time-ray-tracing-engine_amd:$PWD/tests:$PWD
timeout -k 10 500 python -u -m pytest tests/test_multi.py tests/test_persistent.py tests/test_gpu_parity.py tests/test_dist.py tests/test_c5.py tests/test_progressive.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
bash profiles/ab.sh $O/ab.log "C2" "base RTX_TAIL_TILES=0.25 RTX_TAIL_TILES=1 RTX_TAIL_TILES=0" 2 || exit 1
bash profiles/ab.sh $O/ab.log "C3" "base RTX_TAIL_TILES=0 RTX_TAIL_TILES=1 RTX_TAIL_TILES=2" 2 || exit 1
echo done
