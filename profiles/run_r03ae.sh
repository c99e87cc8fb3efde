#!/bin/bash
# r03ae: the uniform split's last tiles in 8x finer chunks (C4: 5 -> 40 chunks, C5: 2 -> 16 for the
# last 2,048 tiles): plan-sensitive GPU tests, then C4/C5 A/B against the plain uniform split
# (base)
set -o pipefail
O=gpurun_out/r03ae
mkdir -p $O
export PYTHONPATH=$PWD/real-time-ray-tracing-engine_amd:$PWD/tests:$PWD
RTX_UNIFORM_TAIL=1 timeout -k 10 500 python -u -m pytest tests/test_c5.py tests/test_multi.py tests/test_persistent.py tests/test_gpu_parity.py tests/test_progressive.py -x -q -m gpu --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
bash profiles/ab.sh $O/ab.log "C4 C5" "RTX_UNIFORM_TAIL=1 base" 2 || exit 1
echo done
