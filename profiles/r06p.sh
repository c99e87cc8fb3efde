#!/bin/bash
# r06p: flat-walk sphere cull (build_dbgF = -DRT_FLAT_CULL=1: a wave skips a flat-list
# sphere every lane's fp32 discriminant bound calls a miss) vs base on C2; bit-identity
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06p
mkdir -p $O
B=$PWD/real-time-ray-tracing-engine_amd/build/librtx_hip.so
F=$PWD/real-time-ray-tracing-engine_amd/build_dbgF/librtx_hip.so
RTX_LIB=$B timeout -k 10 200 python tools/frame_dump.py --config C2 --out /tmp/r06p_base.npy || exit 1
RTX_LIB=$F timeout -k 10 200 python tools/frame_dump.py --config C2 --out /tmp/r06p_F.npy || exit 1
python tools/frame_dump.py --compare /tmp/r06p_base.npy /tmp/r06p_F.npy | tee $O/bitcmp_C2.log
bash profiles/ab.sh $O/ab_C2.log "C2" "base F" 4 || exit 1
echo done
