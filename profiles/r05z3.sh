#!/bin/bash
# r05z3: C3's head units with cost-ordered dispatch on: 128 strata (default),
# whole 256-strata tiles, 64; and the tail share
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05z3
mkdir -p $O
bash profiles/ab.sh $O/ab.log "C3" "base RTX_TUNING=head_strata=256 RTX_TUNING=head_strata=64 RTX_TUNING=tail_tiles=0.125 RTX_TUNING=tail_tiles=0.5" 2 || exit 1
