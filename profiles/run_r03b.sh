#!/bin/bash
# r03b: persistent instance as one 16-wave block per CU (one LDS copy of the BVH per CU: C3's
# whole tree staged) vs r03a's 4-wave blocks (build_dbgR03A): persistence + parity tests, C3/C5 A/B
set -o pipefail
O=gpurun_out/r03b
mkdir -p $O
export PYTHONPATH=$PWD/real-time-ray-tracing-engine_amd:$PWD/tests:$PWD
timeout -k 10 400 python -u -m pytest tests/test_persistent.py tests/test_gpu_parity.py tests/test_c5.py tests/test_bvh4.py -x -v -m gpu --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
python - <<'PY' > $O/info.log 2>&1
import os, sys
from rtx.render import Renderer
from rtx.scene import load_scene
S = load_scene("real-time-ray-tracing-engine_amd/scenes/bouncing_seed42.json")
with Renderer(S) as R:
    print(R.info())
PY
cat $O/info.log
for r in 1 2 3; do
  for v in base R03A; do
    if [ $v = base ]; then L=$PWD/real-time-ray-tracing-engine_amd/build/librtx_hip.so; else L=$PWD/real-time-ray-tracing-engine_amd/build_dbg$v/librtx_hip.so; fi
    RTX_LIB=$L timeout -k 10 200 python bench.py --config C3 --steps 4 --warmup 1 --no-cpu-baseline --pmc off --no-other-configs 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$v', 'C3', d['value'], d['roofline']['kernel_ms'])" || exit 1
  done
done | tee $O/ab.log
for v in base R03A; do
  if [ $v = base ]; then L=$PWD/real-time-ray-tracing-engine_amd/build/librtx_hip.so; else L=$PWD/real-time-ray-tracing-engine_amd/build_dbg$v/librtx_hip.so; fi
  RTX_LIB=$L timeout -k 10 200 python bench.py --config C5 --steps 1 --warmup 1 --no-cpu-baseline --pmc off --no-other-configs 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$v', 'C5', d['value'], d['roofline']['kernel_ms'])" || exit 1
done | tee -a $O/ab.log
echo done
