#!/bin/bash
# r05s: binary vs 4-wide world BVH on this build (C3 scene + 20k random spheres)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05s
mkdir -p $O
timeout -k 10 400 python tools/arity_ab.py --n 5000 20000 --rounds 3 > $O/arity_ab.log 2>&1 || { tail -20 $O/arity_ab.log; exit 1; }
cat $O/arity_ab.log
