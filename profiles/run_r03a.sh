#!/bin/bash
# r03a: round-3 first build (ABI v2, LDS-fit check for 4-wide collapses, bench line: fp64 roofline,
# C3 live PMC, C5 entry, host-output rate, progressive fps, quota-sized CPU baseline, N>1 rank
# diagnostics; new C5 GPU tests) -- full GPU suite, then the default bench line
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03a
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 500 python bench.py > $O/bench_default.log 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
tail -1 $O/bench_default.log | cut -c1-600
echo done
