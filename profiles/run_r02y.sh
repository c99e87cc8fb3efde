#!/bin/bash
# r02y: leaf tests compacted across the wave (ballot prefix + LDS table +
# ds_bpermute ray borrow) = base vs the per-lane leaf loop (L0): parity of every
# BVH instance, C2/C3/C4 A/B, C3 lane utilisation
set -o pipefail
O=gpurun_out/r02y
mkdir -p $O
export PYTHONPATH=$PWD/real-time-ray-tracing-engine_amd:$PWD/tests:$PWD
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_instances.py tests/test_bvh4.py tests/test_device_bvh.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
bash profiles/ab_variants.sh base L0 base L0 > $O/ab.log 2>&1 || exit 1
cat $O/ab.log
timeout -k 10 200 python bench.py --config C3 --steps 2 --warmup 1 --no-cpu-baseline --pmc off --no-other-configs > $O/bench_C3.json 2> $O/bench_C3.err || exit 1
python -c "import json; d=json.loads(open('$O/bench_C3.json').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['lane_utilisation'] if 'lane_utilisation' in d['roofline'] else d.get('lane_utilisation'))"
