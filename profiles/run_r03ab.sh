#!/bin/bash
# r03ab: C2 tail size re-measured on the final build (RTX_TAIL_TILES: tail tiles per wave slot, 0.5 default)
set -o pipefail
O=gpurun_out/r03ab
mkdir -p $O
bash profiles/ab.sh $O/ab.log "C2" "base RTX_TAIL_TILES=0.25 RTX_TAIL_TILES=0.75 RTX_TAIL_TILES=1" 3 || exit 1
echo done
