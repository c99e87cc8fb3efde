#!/bin/bash
# r02am: SAH centroid bins per axis for C3 (host builder; RT_SAH_BINS)
set -o pipefail
O=gpurun_out/r02am
mkdir -p $O
run() { env "$@" timeout -k 10 200 python bench.py --config C3 --steps 3 --warmup 1 --no-cpu-baseline --pmc off --no-other-configs 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$*', 'C3', d['value'])"; }
for r in 1 2; do
  for b in 16 8 32 64; do run RT_SAH_BINS=$b || exit 1; done
done | tee $O/sweep.log
