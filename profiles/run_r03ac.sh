#!/bin/bash
# r03ac: tail chunk split re-measured (RTX_TAIL_SPLIT: tail chunks per head chunk, 8 default) on C2 and C3
set -o pipefail
O=gpurun_out/r03ac
mkdir -p $O
bash profiles/ab.sh $O/ab.log "C2 C3" "base RTX_TAIL_SPLIT=4 RTX_TAIL_SPLIT=16" 2 || exit 1
echo done
