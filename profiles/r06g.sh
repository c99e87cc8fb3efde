#!/bin/bash
# r06g: the traversal stack's top entry held in a register (build_dbgT =
# -DRT_TOS_REG=1) vs base on C3 / C5; C3 frame bit-identity
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06g
mkdir -p $O
B=$PWD/real-time-ray-tracing-engine_amd/build/librtx_hip.so
T=$PWD/real-time-ray-tracing-engine_amd/build_dbgT/librtx_hip.so
RTX_LIB=$B timeout -k 10 200 python tools/frame_dump.py --config C3 --out /tmp/r06g_base.npy || exit 1
RTX_LIB=$T timeout -k 10 200 python tools/frame_dump.py --config C3 --out /tmp/r06g_T.npy || exit 1
python tools/frame_dump.py --compare /tmp/r06g_base.npy /tmp/r06g_T.npy | tee $O/bitcmp_C3.log
bash profiles/ab.sh $O/ab_C3.log "C3" "base T" 3 || exit 1
bash profiles/ab.sh $O/ab_C5.log "C5" "base T" 1 || exit 1
echo done
