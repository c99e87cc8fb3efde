#!/bin/bash
# r03c: base = persistent 16-wave blocks + binary node visit with the slab verdict apart from the
# entry distance and cl32 clamp via v_min3 (40 -> 36 VALU in the visit block) + camera read
# afresh only at path regeneration in the rich instances; R03A = round-3 start; CF0 = base
# without the camera re-read; LP = base + world items and spheres staged in LDS by the
# persistent instance.  Parity (base, and LP on the persistent paths), then C3/C4/C5 A/B.
set -o pipefail
O=gpurun_out/r03c
mkdir -p $O
export PYTHONPATH=$PWD/real-time-ray-tracing-engine_amd:$PWD/tests:$PWD
timeout -k 10 400 python -u -m pytest tests/test_gpu_instances.py tests/test_persistent.py tests/test_gpu_parity.py tests/test_bvh4.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
RTX_LIB=$PWD/real-time-ray-tracing-engine_amd/build_dbgLP/librtx_hip.so timeout -k 10 400 python -u -m pytest tests/test_persistent.py tests/test_gpu_parity.py tests/test_c5.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/gpu_tests_lp.log 2>&1 || { tail -30 $O/gpu_tests_lp.log; exit 1; }
tail -1 $O/gpu_tests_lp.log
RTX_LIB=$PWD/real-time-ray-tracing-engine_amd/build_dbgLP/librtx_hip.so python -c "
from rtx.render import Renderer
from rtx.scene import load_scene
with Renderer(load_scene('real-time-ray-tracing-engine_amd/scenes/bouncing_seed42.json')) as R:
    print(R.info())
" 2>&1 | tail -1
bash profiles/ab.sh $O/ab.log "C3" "base R03A LP" 2 || exit 1
bash profiles/ab.sh $O/ab.log "C4" "base CF0" 2 || exit 1
bash profiles/ab.sh $O/ab.log "C5" "base LP" 1 || exit 1
echo done
