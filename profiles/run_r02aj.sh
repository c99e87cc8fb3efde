#!/bin/bash
# r02aj: host SAH leaf rules for C3 (486 spheres): leaf-max (always-leaf count),
# leaf-split bound and traversal cost (x4) -- measurement overrides
set -o pipefail
O=gpurun_out/r02aj
mkdir -p $O
run() { env "$@" timeout -k 10 200 python bench.py --config C3 --steps 3 --warmup 1 --no-cpu-baseline --pmc off --no-other-configs 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$*', 'C3', d['value'])"; }
for r in 1 2; do
  run RT_SAH_LEAF_MAX=2 || exit 1
  run RT_SAH_LEAF_MAX=1 || exit 1
  run RT_SAH_LEAF_MAX=1 RT_SAH_LEAF_SPLIT=1 || exit 1
  run RT_SAH_LEAF_MAX=3 || exit 1
  run RT_SAH_LEAF_MAX=4 || exit 1
  run RT_SAH_TRAV_X4=2 || exit 1
  run RT_SAH_TRAV_X4=8 || exit 1
  run RT_SAH_LEAF_SPLIT=6 RT_SAH_TRAV_X4=8 || exit 1
done | tee $O/sweep.log
