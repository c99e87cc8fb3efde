#!/bin/bash
# r05z1: C5 (4K spp 4096, persistent BVH instance) with and without tile order
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05z1
mkdir -p $O
bash profiles/ab.sh $O/ab.log "C5" "base RTX_TUNING=no_tile_order=1" 2 || exit 1
