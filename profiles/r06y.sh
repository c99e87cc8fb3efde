#!/bin/bash
# r06y: where r06x's gain comes from -- build/ (plain instances re-measure and re-sort
# every launch), build_dbgP (every instance: the probe's order once per shape, no cost
# atomics compiled), build_dbgH (-DRT_ORDER_ONCE: the plain instances measure costs in
# their first launch of a shape only, then keep that order; atomics compiled, skipped)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06y
mkdir -p $O
B=$PWD/real-time-ray-tracing-engine_amd/build/librtx_hip.so
P=$PWD/real-time-ray-tracing-engine_amd/build_dbgP/librtx_hip.so
H=$PWD/real-time-ray-tracing-engine_amd/build_dbgH/librtx_hip.so
RTX_LIB=$H timeout -k 10 200 python tools/frame_dump.py --config C3 --width 480 --spp 64 --out /tmp/r06y_H.npy || exit 1
RTX_LIB=$B timeout -k 10 200 python tools/frame_dump.py --config C3 --width 480 --spp 64 --out /tmp/r06y_B.npy || exit 1
python tools/frame_dump.py --compare /tmp/r06y_B.npy /tmp/r06y_H.npy | tee $O/bitcmp_C3.log
run() { # label lib config steps warmup
  RTX_LIB=$2 timeout -k 10 200 python bench.py --config $3 --steps $4 --warmup $5 --no-cpu-baseline --pmc off --no-other-configs 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$1', '$3', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], flush=True)"
}
for r in 1 2 3; do
  run base $B C2 20 5 || exit 1
  run P $P C2 20 5 || exit 1
  run H $H C2 20 5 || exit 1
done 2>&1 | tee $O/ab_C2.log
for r in 1 2; do
  run base $B C3 4 1 || exit 1
  run P $P C3 4 1 || exit 1
  run H $H C3 4 1 || exit 1
done 2>&1 | tee $O/ab_C3.log
run base $B C5 1 1 2>&1 | tee $O/ab_C5.log || exit 1
run P $P C5 1 1 2>&1 | tee -a $O/ab_C5.log || exit 1
echo done
