#!/bin/bash
# r04e: deferred fog albedos (RT_DEFER_NOISE) -- the noise / parity GPU tests, then C4 A/B against
# build_dbgD0 (RT_DEFER_NOISE=0, immediate noise), and C3 with the binary walk's signed visit
# restricted to fully staged trees (base vs build_dbgS0)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04e
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_noise_defer.py tests/test_gpu_instances.py tests/test_gpu_parity.py tests/test_statistical_parity.py -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash profiles/ab.sh $O/noise_defer_ab.log "C4" "D0 base" 3 || exit 1
bash profiles/ab.sh $O/c3_ab.log "C3" "S0 base" 2 || exit 1
timeout -k 10 300 python bench.py --config C4 --steps 1 --warmup 1 --no-cpu-baseline --no-other-configs --pmc off > $O/bench_C4_stats.json 2> $O/bench_C4_stats.err || { tail -20 $O/bench_C4_stats.err; exit 1; }
echo done
