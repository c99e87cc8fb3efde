# Rehearse the N>1 bench path on ONE GPU: 2 ranks share cuda:0 and gloo stands in
# for RCCL (tile gather, then stratum reduce); --check compares rank 0's frame
# with a single-device render of all strata.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 300 python bench.py --config C2 --steps 3 --warmup 1 --no-cpu-baseline --check > $O/rehearse_n1.log 2>&1
tail -1 $O/rehearse_n1.log
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --config C2 --steps 3 --warmup 1 --backend gloo --share-device --check > $O/rehearse_n2.log 2>&1
tail -1 $O/rehearse_n2.log
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29519 bench.py --gpus 2 --config C2 --steps 3 --warmup 1 --backend gloo --share-device --check --shard strata > $O/rehearse_n2s.log 2>&1
tail -1 $O/rehearse_n2s.log
