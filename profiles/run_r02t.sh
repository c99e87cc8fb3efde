#!/bin/bash
# r02t: bench lines with live PMC passes for C2, C3 and C4 on the current build;
# the PMC summaries become the committed fallbacks profiles/pmc_<config>.json
set -o pipefail
O=gpurun_out/r02t
mkdir -p $O
export TMPDIR=/tmp
for c in C2 C3 C4; do
  timeout -k 10 500 python bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline --no-other-configs --pmc-save $O/pmc_$c.json > $O/bench_$c.json 2> $O/bench_$c.err || exit 1
done
