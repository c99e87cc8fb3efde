#!/bin/bash
# r02an: idle lanes that trigger a refill in the plain BVH instances
# (RT_REGEN_PLAIN 16 = base, 8, 32) after the persistent waves and
# single-item leaves: C3 A/B
set -o pipefail
O=gpurun_out/r02an
mkdir -p $O
for r in 1 2; do
  for v in base R8 R32; do
    if [ $v = base ]; then L=$PWD/real-time-ray-tracing-engine_amd/build/librtx_hip.so; else L=$PWD/real-time-ray-tracing-engine_amd/build_dbg$v/librtx_hip.so; fi
    RTX_LIB=$L timeout -k 10 200 python bench.py --config C3 --steps 3 --warmup 1 --no-cpu-baseline --pmc off --no-other-configs 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$v', 'C3', d['value'])" || exit 1
  done
done | tee $O/ab.log
