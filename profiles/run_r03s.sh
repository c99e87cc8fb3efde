#!/bin/bash
# r03s: Perlin octave loop software-pipelined (the next octave's cell and permutation reads
# issued while this octave blends; same arithmetic): noise-instance parity, then C4 A/B
# against the plain rolled loop (TP0)
set -o pipefail
O=gpurun_out/r03s
mkdir -p $O
export PYTHONPATH=$PWD/real-time-ray-tracing-engine_amd:$PWD/tests:$PWD
timeout -k 10 400 python -u -m pytest tests/test_lds_perlin.py tests/test_gpu_instances.py tests/test_gpu_parity.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
bash profiles/ab.sh $O/ab.log "C4" "base TP0" 3 || exit 1
echo done
