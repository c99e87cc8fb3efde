#!/bin/bash
# r03l: the epilogue's launch fields / camera width+scale / output pointer read afresh from
# the kernarg segment in every instance (base; C4 instance SGPR spills 150 -> 141) vs held
# across the path loop (EP0).  Instance parity, then C2/C4 A/B.
set -o pipefail
O=gpurun_out/r03l
mkdir -p $O
export PYTHONPATH=$PWD/real-time-ray-tracing-engine_amd:$PWD/tests:$PWD
timeout -k 10 400 python -u -m pytest tests/test_gpu_instances.py tests/test_gpu_parity.py tests/test_multi.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
bash profiles/ab.sh $O/ab.log "C2 C4" "base EP0" 3 || exit 1
echo done
