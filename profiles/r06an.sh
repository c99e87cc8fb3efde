#!/bin/bash
# r06an: the round's last tree (comment-only source changes since r06zz): GPU suite + smoke
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06an
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
echo done
