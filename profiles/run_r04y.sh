#!/bin/bash
# r04y: the persistent tests incl. the staged-tree forms (whole DNodeL tree / prefix / none: bit-identical)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04y
mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu tests/test_persistent.py > $O/persistent.log 2>&1 || { tail -40 $O/persistent.log; exit 1; }
tail -3 $O/persistent.log
echo done
