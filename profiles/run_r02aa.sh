#!/bin/bash
# r02aa: full GPU suite with the product build (per-lane leaf loop) and the
# leaf-share variant check (tests/test_leaf_share.py)
set -o pipefail
O=gpurun_out/r02aa
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 420 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
timeout -k 10 300 python -u -m pytest tests/test_leaf_share.py -m gpu -q -s --timeout 300 --timeout-method thread > $O/leaf_share.log 2>&1 || { tail -30 $O/leaf_share.log; exit 1; }
cat $O/leaf_share.log
