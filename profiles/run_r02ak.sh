#!/bin/bash
# r02ak: single-item leaves for binary-walk scenes (< 4096 items; new default)
# vs the previous 2 / 4 leaf rules (OLD: RT_SAH_LEAF_MAX=2 RT_SAH_LEAF_SPLIT=4):
# full GPU suite, C3 A/B, random-sphere scenes of 1k / 3k through both arities
set -o pipefail
O=gpurun_out/r02ak
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 420 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
run() { env "$@" timeout -k 10 200 python bench.py --config C3 --steps 3 --warmup 1 --no-cpu-baseline --pmc off --no-other-configs 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$*', 'C3', d['value'])"; }
for r in 1 2; do
  run RT_X=new || exit 1
  run RT_SAH_LEAF_MAX=2 RT_SAH_LEAF_SPLIT=4 || exit 1
done | tee $O/ab.log
echo new > $O/arity.log
timeout -k 10 300 python tools/arity_ab.py --n 1000 3000 --rounds 3 --no-c3 >> $O/arity.log 2>&1 || exit 1
echo old >> $O/arity.log
RT_SAH_LEAF_MAX=2 RT_SAH_LEAF_SPLIT=4 timeout -k 10 300 python tools/arity_ab.py --n 1000 3000 --rounds 3 --no-c3 >> $O/arity.log 2>&1 || exit 1
cat $O/arity.log | cut -c1-250
