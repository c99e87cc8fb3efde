#!/bin/bash
# r05k: 8-way shard predictions on this build (C2, C3) with the gather priced and
# rank 0's path-trip lane use; the default bench line
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05k
mkdir -p $O
timeout -k 10 400 python tools/shard_sim.py --config C2 --n 1 8 --units 16384 32768 65536 > $O/shard_sim_C2.log 2>&1 || { tail -5 $O/shard_sim_C2.log; exit 1; }
timeout -k 10 400 python tools/shard_sim.py --config C3 --n 1 8 > $O/shard_sim_C3.log 2>&1 || { tail -5 $O/shard_sim_C3.log; exit 1; }
timeout -k 10 600 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -5 $O/bench_default.err; exit 1; }
echo done
