#!/bin/bash
# r02z: compacted leaf tests only when they take fewer rounds than the per-lane
# loop (L2) vs the per-lane loop (L0): parity of the L2 build, C2/C3/C4 A/B
set -o pipefail
O=gpurun_out/r02z
mkdir -p $O
export PYTHONPATH=$PWD/real-time-ray-tracing-engine_amd:$PWD/tests:$PWD
RTX_LIB=$PWD/real-time-ray-tracing-engine_amd/build_dbgL2/librtx_hip.so timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_instances.py tests/test_bvh4.py tests/test_device_bvh.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
bash profiles/ab_variants.sh L2 L0 L2 L0 > $O/ab.log 2>&1 || exit 1
cat $O/ab.log
RTX_LIB=$PWD/real-time-ray-tracing-engine_amd/build_dbgL2/librtx_hip.so timeout -k 10 200 python bench.py --config C3 --steps 2 --warmup 1 --no-cpu-baseline --pmc off --no-other-configs > $O/bench_C3.json 2> $O/bench_C3.err || exit 1
python -c "import json; d=json.loads(open('$O/bench_C3.json').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['lane_utilisation'])"
