#!/bin/bash
# r06s: cost-ordered dispatch in the rich instance from a probe (build_dbgN: every
# instance maps units through the order; the rich ones get it from one STATS-instance
# probe launch per shape) vs the round-6 base, on C4: the default plan, and whole-tile
# heads (fewer chunk partials) with tails of 1/4, 1/2, 1 tile per slot
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06s
mkdir -p $O
B=$PWD/real-time-ray-tracing-engine_amd/build/librtx_hip.so
N=$PWD/real-time-ray-tracing-engine_amd/build_dbgN/librtx_hip.so
RTX_LIB=$B timeout -k 10 200 python tools/frame_dump.py --config C4 --width 480 --spp 64 --out /tmp/r06s_base.npy || exit 1
RTX_LIB=$N timeout -k 10 200 python tools/frame_dump.py --config C4 --width 480 --spp 64 --out /tmp/r06s_N.npy || exit 1
python tools/frame_dump.py --compare /tmp/r06s_base.npy /tmp/r06s_N.npy | tee $O/bitcmp_C4.log
run() { # label lib tuning
  RTX_LIB=$2 RTX_TUNING=$3 timeout -k 10 200 python bench.py --config C4 --steps 2 --warmup 1 --no-cpu-baseline --pmc off --no-other-configs 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$1', 'C4', d['value'], d['roofline']['kernel_ms'], flush=True)"
}
for r in 1 2; do
  run base $B "" || exit 1
  run N $N "" || exit 1
  run N_head1024_tail0.25 $N "head_strata=1024,tail_tiles=0.25" || exit 1
  run N_head1024_tail0.5 $N "head_strata=1024,tail_tiles=0.5" || exit 1
  run N_head1024_tail1 $N "head_strata=1024,tail_tiles=1" || exit 1
done 2>&1 | tee $O/ab_C4.log
echo done
