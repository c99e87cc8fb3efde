#!/bin/bash
# r05z2: EXPERIMENT -- is the end of C2's frame launch short when its tail is
# the cheapest tiles?  Variant R (build_dbgR, -DRT_TAIL_TOP_EXP): the tail is
# the first raster tiles (the sky rows) in plan order; vs the product (tail =
# last raster tiles, cost-ordered) and plan order
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05z2
mkdir -p $O
L=$PWD/real-time-ray-tracing-engine_amd
run() { # label lib tuning
  RTX_LIB=$2 RTX_TUNING=$3 timeout -k 10 200 python bench.py --config C2 --steps 10 --warmup 1 --no-cpu-baseline --pmc off --no-other-configs 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$1', d['value'], d['roofline']['kernel_ms'], flush=True)"
}
for r in 1 2 3; do
  run base $L/build/librtx_hip.so "" || exit 1
  run planorder $L/build/librtx_hip.so "no_tile_order=1" || exit 1
  run top_q $L/build_dbgR/librtx_hip.so "no_tile_order=1" || exit 1
  run top_h $L/build_dbgR/librtx_hip.so "no_tile_order=1,tail_tiles=0.5" || exit 1
  run top_1 $L/build_dbgR/librtx_hip.so "no_tile_order=1,tail_tiles=1.0" || exit 1
  run top_2 $L/build_dbgR/librtx_hip.so "no_tile_order=1,tail_tiles=2.0" || exit 1
done | tee $O/ab.log
