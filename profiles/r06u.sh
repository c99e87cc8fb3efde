#!/bin/bash
# r06u: the probe's strata per tile, 4 (build_dbgN) vs 16 (build_dbgM), on C4 with the
# default plan and with whole-tile heads (tail 1 tile per slot in 4 chunks)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06u
mkdir -p $O
N=$PWD/real-time-ray-tracing-engine_amd/build_dbgN/librtx_hip.so
M=$PWD/real-time-ray-tracing-engine_amd/build_dbgM/librtx_hip.so
run() { # label lib tuning
  RTX_LIB=$2 RTX_TUNING=$3 timeout -k 10 200 python bench.py --config C4 --steps 2 --warmup 1 --no-cpu-baseline --pmc off --no-other-configs 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$1', 'C4', d['value'], d['roofline']['kernel_ms'], flush=True)"
}
for r in 1 2 3; do
  run N4 $N "" || exit 1
  run M16 $M "" || exit 1
  run N4_t1_s4 $N "head_strata=1024,tail_tiles=1,tail_split=4" || exit 1
  run M16_t1_s4 $M "head_strata=1024,tail_tiles=1,tail_split=4" || exit 1
done 2>&1 | tee $O/ab_C4.log
echo done
