#!/bin/bash
# r03d: scalar (s_load) loads of the wave-uniform scene records in the flat list walk
# (base) vs vector loads (NU); product defaults now: persistent 16-wave blocks with the
# world items/spheres in LDS, camera held in SGPRs (no re-read).  Parity of every instance,
# C2/C4 A/B, and the VALU issue-cost microbenchmark.
set -o pipefail
O=gpurun_out/r03d
mkdir -p $O
export PYTHONPATH=$PWD/real-time-ray-tracing-engine_amd:$PWD/tests:$PWD
timeout -k 10 400 python -u -m pytest tests/test_gpu_instances.py tests/test_persistent.py tests/test_gpu_parity.py tests/test_bvh4.py tests/test_edge_cases.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
bash profiles/ab.sh $O/ab.log "C2 C4" "base NU" 3 || exit 1
timeout -k 10 120 real-time-ray-tracing-engine_amd/build_dbgLP/ubench_valu > $O/ubench_valu.log 2>&1 || exit 1
cat $O/ubench_valu.log
echo done
