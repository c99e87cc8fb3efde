#!/bin/bash
# r04q: 8-way tile shards of C2 and C3 on one GPU (tools/shard_sim.py): the stratum-chunk choice
# (work-unit targets 4096 ... 65536; 32768 is bench.py's default)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04q
mkdir -p $O
for c in C2 C3; do
  timeout -k 10 300 python tools/shard_sim.py --config $c --n 8 4 --units 4096 8192 16384 32768 65536 > $O/shard_units_$c.log 2>&1 || { tail -20 $O/shard_units_$c.log; exit 1; }
  grep '^{' $O/shard_units_$c.log | cut -c1-160
done
echo done
