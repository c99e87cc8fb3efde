#!/bin/bash
# r06f: the binary node visit's slab FMAs as v_pk_fma_f32 pairs (build_dbgQ =
# -DRT_PK_SLAB=1) vs base on C3 / C5; C3 frame bit-identity
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06f
mkdir -p $O
B=$PWD/real-time-ray-tracing-engine_amd/build/librtx_hip.so
Q=$PWD/real-time-ray-tracing-engine_amd/build_dbgQ/librtx_hip.so
RTX_LIB=$B timeout -k 10 200 python tools/frame_dump.py --config C3 --out /tmp/r06f_base.npy || exit 1
RTX_LIB=$Q timeout -k 10 200 python tools/frame_dump.py --config C3 --out /tmp/r06f_Q.npy || exit 1
python tools/frame_dump.py --compare /tmp/r06f_base.npy /tmp/r06f_Q.npy | tee $O/bitcmp_C3.log
bash profiles/ab.sh $O/ab_C3.log "C3" "base Q" 3 || exit 1
bash profiles/ab.sh $O/ab_C5.log "C5" "base Q" 1 || exit 1
echo done
