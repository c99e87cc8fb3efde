#!/bin/bash
# r05y: new tail defaults (head/tail plan 0.25 tail tiles per slot, subset
# tails 125 per mille) -- GPU tests of the plan paths, A/B vs the old defaults
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05y
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_tile_order.py tests/test_subset_auto.py tests/test_multi.py tests/test_persistent.py tests/test_gpu_parity.py tests/test_dist.py tests/test_bench_contract.py > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
bash profiles/ab.sh $O/ab.log "C2 C3" "base RTX_TUNING=tail_tiles=0.5" 3 || exit 1
timeout -k 10 600 python tools/shard_sim.py --config C2 --n 2 4 8 --plan auto > $O/sim_C2.log 2>&1 || { tail $O/sim_C2.log; exit 1; }
grep -h config $O/sim_C2.log | cut -c1-330
echo done
