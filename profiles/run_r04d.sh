#!/bin/bash
# r04d: per-rank device time of 1/2/4/8-way splits on one GPU (tools/shard_sim.py: render + the
# library chunk sum per rank + rank 0's device reorder), C2-C5 on the round-4 build
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04d
mkdir -p $O
for c in C2 C3 C4; do
  timeout -k 10 300 python tools/shard_sim.py --config $c > $O/shard_sim_$c.log 2>&1 || { tail -20 $O/shard_sim_$c.log; exit 1; }
  tail -1 $O/shard_sim_$c.log | cut -c1-300
done
timeout -k 10 400 python tools/shard_sim.py --config C5 --reps 2 > $O/shard_sim_C5.log 2>&1 || { tail -20 $O/shard_sim_C5.log; exit 1; }
tail -1 $O/shard_sim_C5.log | cut -c1-300
echo done
