#!/bin/bash
# r05z0: tile order without the LDS unit record (cost = end - start added to
# the tile's counter) -- the touched GPU tests and the C2 / C3 A/B vs plan order
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05z0
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_bvh4.py tests/test_tile_order.py tests/test_subset_auto.py tests/test_multi.py tests/test_persistent.py > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
bash profiles/ab.sh $O/ab.log "C2 C3 C4" "base RTX_TUNING=no_tile_order=1" 3 || exit 1
echo done
