#!/bin/bash
# r05f6: C5's uniform-split tail with tile order on (half slot default vs a quarter / one)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05f6
mkdir -p $O
bash profiles/ab.sh $O/ab.log "C5" "base RTX_TUNING=tail_tiles=0.25 RTX_TUNING=tail_tiles=1.0" 2 || exit 1
