#!/bin/bash
# r05z4: tile order in every instance (variant A, -DRT_ORDER_ALL=1) -- C4 A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05z4
mkdir -p $O
bash profiles/ab.sh $O/ab.log "C4" "base A" 3 || exit 1
