# Compute-only per-rank times of 1/2/4/8-way splits on one GPU (tools/shard_sim.py), current build.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
for c in C2 C3 C4; do
  timeout -k 10 300 python tools/shard_sim.py --config $c > $O/r01i_shard_sim_$c.log 2>&1 || { tail -20 $O/r01i_shard_sim_$c.log; exit 1; }
  tail -4 $O/r01i_shard_sim_$c.log
done
