#!/bin/bash
# r03m: per-rank kernel time of the N-way tile / strata split on one GPU
# (tools/shard_sim.py) for C2, C3, C4 on the round-3 build: what the driver's
# 8-GPU run can reach before the exchange.
set -o pipefail
O=gpurun_out/r03m
mkdir -p $O
export PYTHONPATH=$PWD/real-time-ray-tracing-engine_amd:$PWD/tests:$PWD
for c in C2 C3 C4; do
  timeout -k 10 240 python -u tools/shard_sim.py --config $c > $O/shard_sim_$c.log 2>&1 || { tail -20 $O/shard_sim_$c.log; exit 1; }
  cat $O/shard_sim_$c.log
done
echo done
