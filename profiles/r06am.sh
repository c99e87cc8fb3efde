#!/bin/bash
# r06am: merged shading (one unit vector / sincos / first root for whichever
# material a lane shades) in every non-BVH4 instance (build_dbgM) vs base
# (plain BVH instances only) on C4 / C2; C4 frame bit-compare
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06am
mkdir -p $O
B=$PWD/real-time-ray-tracing-engine_amd/build/librtx_hip.so
V=$PWD/real-time-ray-tracing-engine_amd/build_dbgM/librtx_hip.so
RTX_LIB=$B timeout -k 10 300 python tools/frame_dump.py --config C4 --out /tmp/r06am_base.npy || exit 1
RTX_LIB=$V timeout -k 10 300 python tools/frame_dump.py --config C4 --out /tmp/r06am_M.npy || exit 1
python tools/frame_dump.py --compare /tmp/r06am_base.npy /tmp/r06am_M.npy | tee $O/bitcmp_C4.log
bash profiles/ab.sh $O/ab_C4.log "C4" "base M" 3 || exit 1
bash profiles/ab.sh $O/ab_C2.log "C2" "base M" 2 || exit 1
echo done
