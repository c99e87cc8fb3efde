#!/bin/bash
# r03ag: the uniform split's tail re-measured on C4/C5 (tail split 16 instead of 8; 1 tail tile per wave slot instead of 0.5)
set -o pipefail
O=gpurun_out/r03ag
mkdir -p $O
bash profiles/ab.sh $O/ab.log "C4 C5" "base RTX_TAIL_SPLIT=16 RTX_TAIL_TILES=1" 2 || exit 1
echo done
