#!/bin/bash
# r04v: 8-way tile shards of C4 and C5 on one GPU: stratum-chunk choice (work-unit targets)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04v
mkdir -p $O
timeout -k 10 400 python tools/shard_sim.py --config C4 --n 8 --units 32768 65536 131072 --reps 2 > $O/shard_units_C4.log 2>&1 || { tail -20 $O/shard_units_C4.log; exit 1; }
grep '^{' $O/shard_units_C4.log | cut -c1-140
timeout -k 10 600 python tools/shard_sim.py --config C5 --n 8 --units 32768 131072 --reps 1 > $O/shard_units_C5.log 2>&1 || { tail -20 $O/shard_units_C5.log; exit 1; }
grep '^{' $O/shard_units_C5.log | cut -c1-140
echo done
