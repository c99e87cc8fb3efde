#!/bin/bash
# r06al: one refill site in the flat instance (build_dbgO: the lanes idle after a
# trace take their next items there; one philox10 per lane draws the hit lanes'
# shading block and the refilled lanes' camera block; no refill at the trip's top)
# vs base on C2; frame comparison; GPU parity tests on O
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06al
mkdir -p $O
B=$PWD/real-time-ray-tracing-engine_amd/build/librtx_hip.so
V=$PWD/real-time-ray-tracing-engine_amd/build_dbgO/librtx_hip.so
RTX_LIB=$B timeout -k 10 200 python tools/frame_dump.py --config C2 --out /tmp/r06al_base.npy || exit 1
RTX_LIB=$V timeout -k 10 200 python tools/frame_dump.py --config C2 --out /tmp/r06al_O.npy || exit 1
python tools/frame_dump.py --compare /tmp/r06al_base.npy /tmp/r06al_O.npy | tee $O/cmp_C2.log
bash profiles/ab.sh $O/ab_C2.log "C2" "base O" 4 || exit 1
RTX_LIB=$V timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_instances.py tests/test_multi.py tests/test_tile_order.py tests/test_subset_auto.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests_O.log 2>&1 || { tail -30 $O/gpu_tests_O.log; exit 1; }
tail -1 $O/gpu_tests_O.log
echo done
