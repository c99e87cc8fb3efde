#!/bin/bash
# r06aa: every instance takes its order from the probe (build/): GPU suite + smoke; the
# probe's size on C2 (probe_strata 1 / 4 / 16) A/B; a one-shot render's probe cost;
# progressive frames ordered (build_dbgQ)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06aa
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for c in C2 C3 C4; do timeout -k 10 200 python tools/probe_cost.py --config $c --probe 1 4 16 || exit 1; done 2>&1 | tee $O/probe_cost.log
run() { # label config steps warmup tuning
  RTX_TUNING=$5 timeout -k 10 200 python bench.py --config $2 --steps $3 --warmup $4 --no-cpu-baseline --pmc off --no-other-configs 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$1', '$2', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], flush=True)"
}
for r in 1 2 3; do
  run p16 C2 20 5 "" || exit 1
  run p4 C2 20 5 "probe_strata=4" || exit 1
  run p1 C2 20 5 "probe_strata=1" || exit 1
done 2>&1 | tee $O/ab_C2.log
for r in 1 2; do
  run p16 C3 4 1 "" || exit 1
  run p4 C3 4 1 "probe_strata=4" || exit 1
  run p16 C4 2 1 "" || exit 1
done 2>&1 | tee $O/ab_C3_C4.log
# ordering one-stratum (progressive) launches too (build_dbgQ: kOrderMinStrata 1): the
# progressive device frame rates, build/ vs build_dbgQ
prog() { # label lib
  RTX_LIB=$2 timeout -k 10 200 python -c "
import torch, bench
r = bench.progressive_rates(torch, torch.device('cuda', 0))
print('$1', {c: (v['device_ms_per_frame'], v['display_ms_per_frame']) for c, v in r.items()}, flush=True)" 2>/dev/null
}
Q=$PWD/real-time-ray-tracing-engine_amd/build_dbgQ/librtx_hip.so
B=$PWD/real-time-ray-tracing-engine_amd/build/librtx_hip.so
for r in 1 2 3; do prog base $B || exit 1; prog Q $Q || exit 1; done 2>&1 | tee $O/ab_progressive.log
echo done
