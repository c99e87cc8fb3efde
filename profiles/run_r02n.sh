#!/bin/bash
# r02n: deferred medium record + sin_n for the noise texture (base) vs the
# library sin (S0): GPU parity of base, then C2/C3/C4 A/B interleaved.
set -o pipefail
O=gpurun_out/r02n
mkdir -p $O
export PYTHONPATH=$PWD/real-time-ray-tracing-engine_amd
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_instances.py tests/test_bvh4.py tests/test_statistical_parity.py tests/test_stored_form.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
bash profiles/ab_variants.sh base S0 base S0 > $O/ab.log 2>&1
