#!/bin/bash
# r06ap: the binary walk leaves its node loop for the leaf tests once fewer than K
# walking lanes still lack a leaf and one holds a leaf (build_dbgK<K>,
# RT_LEAF_EXIT_K; base K = 1: every walking lane holds one) -- a short C3 run per
# variant first, then C3 frame bit-compare for K = 4 and C3 A/B for K = 4 / 8
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06ap
mkdir -p $O
B=$PWD/real-time-ray-tracing-engine_amd/build/librtx_hip.so
for k in 4 8; do
  RTX_LIB=$PWD/real-time-ray-tracing-engine_amd/build_dbgK$k/librtx_hip.so timeout -k 5 60 python bench.py --config C3 --width 320 --spp 16 --steps 1 --warmup 1 --no-cpu-baseline --pmc off --no-other-configs > $O/short_K$k.json 2>&1 || { echo "K$k short run failed"; tail -5 $O/short_K$k.json; exit 1; }
  echo "K$k short ok"
done
V=$PWD/real-time-ray-tracing-engine_amd/build_dbgK4/librtx_hip.so
RTX_LIB=$B timeout -k 10 120 python tools/frame_dump.py --config C3 --out /tmp/r06ap_base.npy || exit 1
RTX_LIB=$V timeout -k 10 120 python tools/frame_dump.py --config C3 --out /tmp/r06ap_K4.npy || exit 1
python tools/frame_dump.py --compare /tmp/r06ap_base.npy /tmp/r06ap_K4.npy | tee $O/bitcmp_C3.log
bash profiles/ab.sh $O/ab_C3.log "C3" "base K4 K8" 2 || exit 1
echo done
