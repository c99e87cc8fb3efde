#!/bin/bash
# r05u: cost-ordered dispatch (tile order) -- GPU tests of the touched paths,
# A/B against plan order (RTX_TUNING=no_tile_order=1) and the previous build
# (O), 8-way shares, unit timelines of the ordered launches
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05u
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_tile_order.py tests/test_subset_auto.py tests/test_multi.py tests/test_persistent.py tests/test_c5.py > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
bash profiles/ab.sh $O/ab.log "C2 C3 C4" "base RTX_TUNING=no_tile_order=1 O" 2 || exit 1
timeout -k 10 300 python tools/shard_sim.py --config C2 --n 4 8 --plan auto > $O/sim_C2.log 2>&1 || { tail $O/sim_C2.log; exit 1; }
timeout -k 10 300 python tools/shard_sim.py --config C3 --n 8 --plan auto > $O/sim_C3.log 2>&1 || { tail $O/sim_C3.log; exit 1; }
grep -h '"config"' $O/sim_C*.log | cut -c1-400
echo done
