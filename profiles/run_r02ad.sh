#!/bin/bash
# r02ad: work units per resident wave (RTX_CHUNK_TARGET) for C3 now that its
# waves pull units dynamically
set -o pipefail
O=gpurun_out/r02ad
mkdir -p $O
for r in 1 2; do
  for t in 4 8 16 32 64; do
    RTX_CHUNK_TARGET=$t timeout -k 10 200 python bench.py --config C3 --steps 3 --warmup 1 --no-cpu-baseline --pmc off --no-other-configs 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('target=$t', 'C3', d['value'])" || exit 1
  done
done | tee $O/sweep.log
