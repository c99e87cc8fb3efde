#!/bin/bash
# r06ab: every launch shape ordered by its probe, progressive (one-stratum) frames
# included: GPU suite + smoke, the driver's default line, C4 x3
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06ab
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -1 $O/bench.json | cut -c1-300
for r in 1 2 3; do
  timeout -k 10 200 python bench.py --config C4 --steps 2 --warmup 1 --no-cpu-baseline --pmc off --no-other-configs 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('C4', d['value'], d['roofline']['kernel_ms'], flush=True)" || exit 1
done 2>&1 | tee $O/c4.log
echo done
