#!/bin/bash
# r05f4: the frame tail at an eighth / a sixteenth of the slots (C2, C3)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05f4
mkdir -p $O
bash profiles/ab.sh $O/ab.log "C2 C3" "base RTX_TUNING=tail_tiles=0.125 RTX_TUNING=tail_tiles=0.0625" 3 || exit 1
