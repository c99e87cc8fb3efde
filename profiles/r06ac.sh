#!/bin/bash
# r06ac: larger probes (rt_tuning probe_strata 16 default / 64) on C3, C4 and C2 (where
# 64 = every stratum of the frame)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06ac
mkdir -p $O
run() { # label config steps warmup tuning
  RTX_TUNING=$5 timeout -k 10 200 python bench.py --config $2 --steps $3 --warmup $4 --no-cpu-baseline --pmc off --no-other-configs 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$1', '$2', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], flush=True)"
}
for r in 1 2 3; do
  run p16 C2 20 5 "" || exit 1
  run p64 C2 20 5 "probe_strata=64" || exit 1
  run p16 C3 4 1 "" || exit 1
  run p64 C3 4 1 "probe_strata=64" || exit 1
done 2>&1 | tee $O/ab_C2_C3.log
for r in 1 2; do
  run p16 C4 2 1 "" || exit 1
  run p64 C4 2 1 "probe_strata=64" || exit 1
done 2>&1 | tee $O/ab_C4.log
echo done
