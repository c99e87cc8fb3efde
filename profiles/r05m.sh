#!/bin/bash
# r05m: is the 8-way per-rank spread content or clock history (ranks timed
# forward and reversed, per-rank STATS work); host cost of the N>1 step at an
# 8-way rank's share of C2 (world-of-one pg rehearsal, tile layout, 640 wide
# ~ 1/9 frame; no sync inside the timed loop)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05m
mkdir -p $O
timeout -k 10 300 python tools/shard_sim.py --config C2 --n 8 --units 16384 32768 > $O/shard_warm.log 2>&1 || { tail $O/shard_warm.log; exit 1; }
timeout -k 10 300 python tools/shard_sim.py --config C2 --n 8 --units 32768 --rank-order rev > $O/shard_warm_rev.log 2>&1 || { tail $O/shard_warm_rev.log; exit 1; }
for w in 640 1920; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29531 bench.py --config C2 --width $w --steps 60 --warmup 5 --pg-rehearsal --no-cpu-baseline --pmc off --no-other-configs > $O/reh_$w.json 2> $O/reh_$w.err || { tail $O/reh_$w.err; exit 1; }
done
grep -h '"config"' $O/shard_*.log
for f in $O/reh*.json; do python -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['value'], d['ms_per_step'], d['host_issue_ms_per_step'], d['ranks']['per_rank_kernel_ms'], d['ranks']['exchange_ms_rank0'], d['config']['parallelism'])"; done
