#!/bin/bash
# r03o: re-entry check of HEAD (3ee9951) on a fresh box -- full GPU suite and the default
# (driver) bench line, C4 with its live PMC passes (VALU busy after the LDS Perlin table)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03o
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 600 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
tail -1 $O/bench_default.json | cut -c1-400
timeout -k 10 400 python bench.py --config C4 --steps 2 --warmup 1 --no-cpu-baseline --no-other-configs --pmc-save $O/pmc_C4.json > $O/bench_C4.json 2> $O/bench_C4.err || { tail -20 $O/bench_C4.err; exit 1; }
tail -1 $O/bench_C4.json | cut -c1-300
echo done
