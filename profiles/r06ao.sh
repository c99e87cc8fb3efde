#!/bin/bash
# r06ao: Philox round keys derived in VGPRs at each call (an asm "+v" barrier on
# the seed: 18 v_add per block instead of the hoisted round keys' SGPR spills and
# v_readlanes): build_dbgV in the rich instances, build_dbgW also in the plain BVH
# instances; vs base on C4 / C3 / C5; C4 and C3 frame bit-compare
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06ao
mkdir -p $O
B=$PWD/real-time-ray-tracing-engine_amd/build/librtx_hip.so
V=$PWD/real-time-ray-tracing-engine_amd/build_dbgV/librtx_hip.so
W=$PWD/real-time-ray-tracing-engine_amd/build_dbgW/librtx_hip.so
RTX_LIB=$B timeout -k 10 300 python tools/frame_dump.py --config C4 --out /tmp/r06ao_base4.npy || exit 1
RTX_LIB=$V timeout -k 10 300 python tools/frame_dump.py --config C4 --out /tmp/r06ao_V4.npy || exit 1
python tools/frame_dump.py --compare /tmp/r06ao_base4.npy /tmp/r06ao_V4.npy | tee $O/bitcmp_C4.log
RTX_LIB=$B timeout -k 10 300 python tools/frame_dump.py --config C3 --out /tmp/r06ao_base3.npy || exit 1
RTX_LIB=$W timeout -k 10 300 python tools/frame_dump.py --config C3 --out /tmp/r06ao_W3.npy || exit 1
python tools/frame_dump.py --compare /tmp/r06ao_base3.npy /tmp/r06ao_W3.npy | tee $O/bitcmp_C3.log
bash profiles/ab.sh $O/ab_C4.log "C4" "base V" 3 || exit 1
bash profiles/ab.sh $O/ab_C3.log "C3" "base W" 2 || exit 1
bash profiles/ab.sh $O/ab_C5.log "C5" "base W" 1 || exit 1
echo done
