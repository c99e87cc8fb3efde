#!/bin/bash
# r04a: round-4 start (dead-switch cleanup, device tile exchange) -- full GPU suite, smoke,
# the default (driver) bench line, the rt_multi exchange timing, the counter list and a
# VALU-counter calibration on the microbenchmark
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04a
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
cat $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
tail -1 $O/bench_default.json | cut -c1-400
timeout -k 10 300 python tools/multi_gather.py --config C2 --shards 2 4 8 > $O/multi_gather_C2.log 2>&1 || { tail -20 $O/multi_gather_C2.log; exit 1; }
cat $O/multi_gather_C2.log
timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1 || { tail -5 $O/counters.txt; exit 1; }
C=""
for c in SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE; do
  if grep -qw "$c" $O/counters.txt; then C="$C $c"; fi
done
echo "pmc:$C"
timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/ubench_pmc -o ub -- real-time-ray-tracing-engine_amd/build/ubench_issue > $O/ubench_pmc.log 2>&1 || { tail -20 $O/ubench_pmc.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ubench_trace -o ub -- real-time-ray-tracing-engine_amd/build/ubench_issue > $O/ubench_trace.log 2>&1 || { tail -20 $O/ubench_trace.log; exit 1; }
timeout -k 10 60 real-time-ray-tracing-engine_amd/build/ubench_issue > $O/ubench_issue.log 2>&1 || exit 1
cat $O/ubench_issue.log
echo done
