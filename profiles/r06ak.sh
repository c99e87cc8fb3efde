#!/bin/bash
# r06ak: fused refill (missed lanes take their next items right after the trace;
# one philox10 draws the hit lanes' shading block and the refilled lanes' camera
# block): build_dbgF in the flat instance (C2), build_dbgG also in the plain BVH
# instances (C3 / C5); frame comparisons; GPU parity tests on G
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06ak
mkdir -p $O
B=$PWD/real-time-ray-tracing-engine_amd/build/librtx_hip.so
G=$PWD/real-time-ray-tracing-engine_amd/build_dbgG/librtx_hip.so
for c in C2 C3; do
  RTX_LIB=$B timeout -k 10 200 python tools/frame_dump.py --config $c --out /tmp/r06ak_base_$c.npy || exit 1
  RTX_LIB=$G timeout -k 10 200 python tools/frame_dump.py --config $c --out /tmp/r06ak_G_$c.npy || exit 1
  python tools/frame_dump.py --compare /tmp/r06ak_base_$c.npy /tmp/r06ak_G_$c.npy | tee $O/cmp_$c.log
done
bash profiles/ab.sh $O/ab_C2.log "C2" "base F G" 3 || exit 1
bash profiles/ab.sh $O/ab_C3.log "C3" "base G" 2 || exit 1
bash profiles/ab.sh $O/ab_C5.log "C5" "base G" 1 || exit 1
RTX_LIB=$G timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_instances.py tests/test_multi.py tests/test_tile_order.py tests/test_persistent.py tests/test_c5.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests_G.log 2>&1 || { tail -30 $O/gpu_tests_G.log; exit 1; }
tail -1 $O/gpu_tests_G.log
echo done
