#!/bin/bash
# r02ai: smoke(), and the N>1 bench path rehearsed on one GPU for the BVH
# config C3 (persistent chunked instance under stratum sharding; tile shards
# one unit per wave), --check against a one-device render
set -o pipefail
O=gpurun_out/r02ai
mkdir -p $O
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
cat $O/smoke.log
for sh in tiles strata; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29521 bench.py --gpus 2 --config C3 --steps 2 --warmup 1 --backend gloo --share-device --check --shard $sh > $O/rehearse_C3_$sh.log 2>&1 || { tail -20 $O/rehearse_C3_$sh.log; exit 1; }
  tail -1 $O/rehearse_C3_$sh.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$sh', d['value'], {k: v for k, v in d.items() if 'check' in k})"
done
