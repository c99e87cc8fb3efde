#!/bin/bash
# r03b: (1) persistent instance as one 16-wave block per CU (one LDS copy of the BVH per CU: C3's
# whole tree staged) and (2) the camera read afresh from the kernarg segment in the rich
# instances (C4 instance SGPR spills 150 -> 72), both vs r03a (build_dbgR03A); (3) variant SF:
# also the scene tables afresh per segment (spills 51).  Parity tests, then C3/C4/C5 A/B.
set -o pipefail
O=gpurun_out/r03b
mkdir -p $O
export PYTHONPATH=$PWD/real-time-ray-tracing-engine_amd:$PWD/tests:$PWD
timeout -k 10 500 python -u -m pytest tests/test_persistent.py tests/test_gpu_parity.py tests/test_gpu_instances.py tests/test_c5.py tests/test_bvh4.py -x -v -m gpu --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
python -c "
from rtx.render import Renderer
from rtx.scene import load_scene
for n in ('bouncing_seed42', 'cornell_fog'):
    with Renderer(load_scene('real-time-ray-tracing-engine_amd/scenes/%s.json' % n)) as R:
        print(n, R.info())
" > $O/info.log 2>&1; cat $O/info.log
bash profiles/ab.sh $O/ab.log "C3 C4" "base R03A SF" 2 || exit 1
bash profiles/ab.sh $O/ab.log "C5" "base R03A" 1 || exit 1
echo done
