#!/bin/bash
# r05z5: tile order only for launches of >= 16 strata -- tests, the default
# bench line (progressive frames back to their pre-order cost)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05z5
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_tile_order.py tests/test_subset_auto.py tests/test_multi.py tests/test_progressive.py > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 600 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
python -c "import json; d=json.loads(open('$O/bench_default.json').read().strip().splitlines()[-1]); print(d['value'], {c: v['value'] for c, v in d['other_configs'].items()}, {c:(v['device_ms_per_frame'], v['display_ms_per_frame']) for c,v in d['progressive'].items()})"
