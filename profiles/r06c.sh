#!/bin/bash
# r06c: the fp32 leaf pre-test (rt_path.h sphere_cull32, build_dbgP = -DRT_LEAF_PRE=1)
# vs base on C3 / C5: interleaved A/B, STATS counters of both, C3 frame bit-identity
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06c
mkdir -p $O
B=$PWD/real-time-ray-tracing-engine_amd/build/librtx_hip.so
P=$PWD/real-time-ray-tracing-engine_amd/build_dbgP/librtx_hip.so
for v in base P; do
  L=$B; [ $v = P ] && L=$P
  RTX_LIB=$L timeout -k 10 200 python tools/frame_dump.py --config C3 --out /tmp/r06c_frame_C3_$v.npy || exit 1
  RTX_LIB=$L timeout -k 10 200 python bench.py --config C3 --steps 2 --warmup 1 --no-cpu-baseline --pmc off --no-other-configs > $O/stats_C3_$v.json || exit 1
done
python tools/frame_dump.py --compare /tmp/r06c_frame_C3_base.npy /tmp/r06c_frame_C3_P.npy | tee $O/bitcmp_C3.log
bash profiles/ab.sh $O/ab_C3.log "C3" "base P" 3 || exit 1
bash profiles/ab.sh $O/ab_C5.log "C5" "base P" 1 || exit 1
echo done
