#!/bin/bash
# r06q: the cost of cost-ordered dispatch's tile mapping alone in the rich instance
# (build_dbgO = -DRT_ORDER_ALL_READ=1: every instance maps units through tile_order, the
# cost atomics stay in the plain instances) -- C4 A/B and bit-identity (480 wide, spp 64)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06q
mkdir -p $O
B=$PWD/real-time-ray-tracing-engine_amd/build/librtx_hip.so
V=$PWD/real-time-ray-tracing-engine_amd/build_dbgO/librtx_hip.so
RTX_LIB=$B timeout -k 10 200 python tools/frame_dump.py --config C4 --width 480 --spp 64 --out /tmp/r06q_base.npy || exit 1
RTX_LIB=$V timeout -k 10 200 python tools/frame_dump.py --config C4 --width 480 --spp 64 --out /tmp/r06q_O.npy || exit 1
python tools/frame_dump.py --compare /tmp/r06q_base.npy /tmp/r06q_O.npy | tee $O/bitcmp_C4.log
bash profiles/ab.sh $O/ab_C4.log "C4" "base O" 3 || exit 1
echo done
