#!/bin/bash
# r04m: C3 A/B -- staged child entries as absolute LDS addresses (base) against byte offsets
# (build_dbgA0, RT_LDS_ABS=0) and the binary visit's push/advance/pop as selects (build_dbgVS,
# RT_VISIT_SELECT=1); the discriminant sqrt without input/output scaling unless a lane needs it
# (base) against build_dbgSD0 (RT_SQRT_D=0) on C2, C3, C4; parity tests of the walk on the base
# and on the select variant
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04m
mkdir -p $O
T="tests/test_gpu_parity.py tests/test_persistent.py tests/test_c5.py tests/test_bvh4.py tests/test_device_bvh.py tests/test_gpu_arith.py"
timeout -k 10 600 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu $T > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
RTX_LIB=$PWD/real-time-ray-tracing-engine_amd/build_dbgVS/librtx_hip.so timeout -k 10 600 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_persistent.py > $O/parity_vs.log 2>&1 || { tail -30 $O/parity_vs.log; exit 1; }
tail -1 $O/parity_vs.log
bash profiles/ab.sh $O/c3_ab.log "C3" "base A0 VS SD0" 3 || exit 1
bash profiles/ab.sh $O/c2_c4_ab.log "C2 C4" "base SD0" 3 || exit 1
echo done
