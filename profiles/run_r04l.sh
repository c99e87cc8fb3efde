#!/bin/bash
# r04l: binary nodes staged in LDS as DNodeL (per axis lo, hi, lo pairs: one ds_read2_b64 per axis,
# inner children as byte offsets) against build_dbgT0 (RT_LDS_TRIPLE=0, DNode as staged):
# C3 x3, C5 x2; the partly staged large trees (tools/arity_ab.py); the walk's parity tests
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04l
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_persistent.py tests/test_c5.py tests/test_bvh4.py tests/test_device_bvh.py tests/test_leaf_share.py > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
bash profiles/ab.sh $O/c3_ab.log "C3" "base T0" 3 || exit 1
bash profiles/ab.sh $O/c5_ab.log "C5" "base T0" 2 || exit 1
for v in T0 base; do
  if [ $v = base ]; then L=$PWD/real-time-ray-tracing-engine_amd/build/librtx_hip.so; else L=$PWD/real-time-ray-tracing-engine_amd/build_dbg$v/librtx_hip.so; fi
  echo "== $v" >> $O/arity_ab.log
  RTX_LIB=$L timeout -k 10 300 python tools/arity_ab.py --n 100000 --rounds 2 >> $O/arity_ab.log 2>&1 || { tail -20 $O/arity_ab.log; exit 1; }
done
grep -v amdgpu.ids $O/arity_ab.log
echo done
