#!/bin/bash
# r06x: every instance takes the probe's order once per shape (build_dbgP =
# -DRT_PROBE_ALL=1: no in-kernel cost atomics, no per-launch memset / sort) vs build/
# (the plain instances re-measure every launch) -- C2 (the driver's command) and C3 A/B,
# C2 bit-compare
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06x
mkdir -p $O
B=$PWD/real-time-ray-tracing-engine_amd/build/librtx_hip.so
P=$PWD/real-time-ray-tracing-engine_amd/build_dbgP/librtx_hip.so
RTX_LIB=$B timeout -k 10 200 python tools/frame_dump.py --config C2 --width 480 --spp 64 --out /tmp/r06x_base.npy || exit 1
RTX_LIB=$P timeout -k 10 200 python tools/frame_dump.py --config C2 --width 480 --spp 64 --out /tmp/r06x_P.npy || exit 1
python tools/frame_dump.py --compare /tmp/r06x_base.npy /tmp/r06x_P.npy | tee $O/bitcmp_C2.log
run() { # label lib config steps warmup
  RTX_LIB=$2 timeout -k 10 200 python bench.py --config $3 --steps $4 --warmup $5 --no-cpu-baseline --pmc off --no-other-configs 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$1', '$3', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], flush=True)"
}
for r in 1 2 3 4; do
  run base $B C2 20 5 || exit 1
  run P $P C2 20 5 || exit 1
done 2>&1 | tee $O/ab_C2.log
for r in 1 2; do
  run base $B C3 4 1 || exit 1
  run P $P C3 4 1 || exit 1
done 2>&1 | tee $O/ab_C3.log
echo done
