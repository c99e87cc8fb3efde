#!/bin/bash
# r03k: child-interleaved DNode planes (lo[axis][child]) and the binary node visit's twelve
# plane FMAs as six v_pk_fma_f32 with op_sel broadcasts of the per-ray constants, the
# entry/exit min/max in asm (no re-canonicalisation): visit block 40 -> 35 VALU.  Base vs SP0
# (same layout, scalar FMAs); Perlin FMA/lerp back on (C4).  BVH/persistence/parity tests.
set -o pipefail
O=gpurun_out/r03k
mkdir -p $O
export PYTHONPATH=$PWD/real-time-ray-tracing-engine_amd:$PWD/tests:$PWD
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_persistent.py tests/test_gpu_instances.py tests/test_bvh4.py tests/test_device_bvh.py tests/test_c5.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
bash profiles/ab.sh $O/ab.log "C3 C4" "base SP0" 3 || exit 1
echo done
