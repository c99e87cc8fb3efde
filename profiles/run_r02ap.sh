#!/bin/bash
# r02ap: final round-2 build (after per-unit kernarg reads, a793c22) -- full GPU suite, default bench line (live PMC
# passes + reference -p CPU baseline), kernel traces of C2 and C3
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02ap
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 420 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 400 python bench.py > $O/bench_default.log 2> $O/bench_default.err || exit 1
tail -1 $O/bench_default.log | cut -c1-400
for c in C2 C3; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$c -o $c -- python bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline --no-other-configs --pmc off > $O/trace_$c.log 2>&1 || exit 1
done
echo done
