#!/bin/bash
# r05f1: final profile set of round 5 -- full GPU suite, the default (driver) bench line,
# PMC summaries (bench.py --pmc-save: VALU / FETCH_SIZE / WRITE_SIZE passes) for C2-C5, and
# rocprofv3 --kernel-trace --stats of C2, C3, C4 (bench.py, 5 steps)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05f1
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
cat $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
tail -1 $O/bench_default.json | cut -c1-300
for c in C4 C5; do
  timeout -k 10 400 python bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline --no-other-configs --pmc-save $O/pmc_$c.json > $O/bench_$c.json 2> $O/bench_$c.err || { tail -20 $O/bench_$c.err; exit 1; }
  tail -1 $O/bench_$c.json | cut -c1-300
done
for c in C2 C3; do
  timeout -k 10 300 python bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-other-configs --pmc-save $O/pmc_$c.json > $O/bench_$c.json 2> $O/bench_$c.err || { tail -20 $O/bench_$c.err; exit 1; }
done
for c in C2 C3 C4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$c -o $c -- python bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline --no-other-configs --pmc off > $O/trace_$c.log 2>&1 || { tail -20 $O/trace_$c.log; exit 1; }
done
find $O -name "*kernel_stats.csv" | head
echo done
