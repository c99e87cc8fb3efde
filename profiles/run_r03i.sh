#!/bin/bash
# r03i: the flat instance's refill threshold (idle lanes before camera rays are generated:
# base 16, RG8, RG32) and occupancy target (WF5: 5 waves/SIMD) re-measured with one-wave
# blocks and whole-tile head units
set -o pipefail
O=gpurun_out/r03i
mkdir -p $O
bash profiles/ab.sh $O/ab.log "C2" "base RG8 RG32 WF5" 3 || exit 1
echo done
