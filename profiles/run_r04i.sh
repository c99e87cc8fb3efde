#!/bin/bash
# r04i: C3 A/B of two parked leaves per lane (build_dbgP2, RT_PARK2=1) against the final build,
# and the variant's C3 STATS line (lane use, node-loop iterations)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04i
mkdir -p $O
bash profiles/ab.sh $O/park2_ab.log "C3" "base P2" 3 || exit 1
RTX_LIB=$PWD/real-time-ray-tracing-engine_amd/build_dbgP2/librtx_hip.so timeout -k 10 300 python bench.py --config C3 --steps 3 --warmup 1 --no-cpu-baseline --no-other-configs --pmc off > $O/bench_C3_stats_p2.json 2> $O/bench_C3_stats_p2.err || { tail -20 $O/bench_C3_stats_p2.err; exit 1; }
RTX_LIB=$PWD/real-time-ray-tracing-engine_amd/build_dbgP2/librtx_hip.so timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_persistent.py > $O/p2_parity.log 2>&1 || { tail -30 $O/p2_parity.log; exit 1; }
tail -1 $O/p2_parity.log
echo done
