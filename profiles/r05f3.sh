#!/bin/bash
# r05f3: C2's frame tail around the new default (a quarter slot, 8x split)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05f3
mkdir -p $O
bash profiles/ab.sh $O/ab.log "C2" "base RTX_TUNING=tail_split=4 RTX_TUNING=tail_tiles=0.125 RTX_TUNING=tail_tiles=0.375 RTX_TUNING=tail_split=12" 3 || exit 1
