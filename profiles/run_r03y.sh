#!/bin/bash
# r03y: the plain BVH instances' refill threshold re-measured after the at-use constants
# (16 idle lanes, base; 8: R8; 24: R24) on C3
set -o pipefail
O=gpurun_out/r03y
mkdir -p $O
bash profiles/ab.sh $O/ab.log "C3" "base R8 R24" 3 || exit 1
echo done
