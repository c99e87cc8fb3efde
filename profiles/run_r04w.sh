#!/bin/bash
# r04w: rehearse the N>1 bench path on ONE GPU (2 ranks share cuda:0, gloo in place of RCCL) on the
# final round-4 build: C2 and C3 tile shards (the strata-scaled unit target) and C2 stratum
# shards, each with --check against a one-device render
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04w
mkdir -p $O
P=29531
for run in "C2 tiles" "C3 tiles" "C2 strata"; do
  set -- $run
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $P bench.py --gpus 2 --config $1 --steps 2 --warmup 1 --backend gloo --share-device --check --shard $2 --no-other-configs > $O/rehearse_$1_$2.log 2>&1 || { tail -30 $O/rehearse_$1_$2.log; exit 1; }
  tail -1 $O/rehearse_$1_$2.log | cut -c1-400
  P=$((P+2))
done
echo done
