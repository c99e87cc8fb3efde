#!/bin/bash
# r06e: Philox round keys from a kernarg table (build_dbgK = -DRT_RK_TABLE=1: philox10
# KB 2 in the rich instances) vs base on C4; C4 frame bit-identity (480 wide, spp 64)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06e
mkdir -p $O
B=$PWD/real-time-ray-tracing-engine_amd/build/librtx_hip.so
K=$PWD/real-time-ray-tracing-engine_amd/build_dbgK/librtx_hip.so
RTX_LIB=$B timeout -k 10 200 python tools/frame_dump.py --config C4 --width 480 --spp 64 --out /tmp/r06e_base.npy || exit 1
RTX_LIB=$K timeout -k 10 200 python tools/frame_dump.py --config C4 --width 480 --spp 64 --out /tmp/r06e_K.npy || exit 1
python tools/frame_dump.py --compare /tmp/r06e_base.npy /tmp/r06e_K.npy | tee $O/bitcmp_C4.log
bash profiles/ab.sh $O/ab_C4.log "C4" "base K" 3 || exit 1
echo done
