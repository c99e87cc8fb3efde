#!/bin/bash
# r02ae: next work unit fetched at unit start (base, RT_UNIT_PREFETCH=1) vs at
# unit end (P0: one register less across the unit): C3 A/B
set -o pipefail
O=gpurun_out/r02ae
mkdir -p $O
for r in 1 2 3; do
  for v in base P0; do
    if [ $v = base ]; then L=$PWD/real-time-ray-tracing-engine_amd/build/librtx_hip.so; else L=$PWD/real-time-ray-tracing-engine_amd/build_dbg$v/librtx_hip.so; fi
    RTX_LIB=$L timeout -k 10 200 python bench.py --config C3 --steps 3 --warmup 1 --no-cpu-baseline --pmc off --no-other-configs 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$v', 'C3', d['value'])" || exit 1
  done
done | tee $O/ab.log
