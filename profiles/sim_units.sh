# Per-rank compute time of 8-way tile shards vs work-unit target (tools/shard_sim.py).
set -e
for u in 16384 32768 65536 131072; do
  RTX_SHARD_UNITS=$u timeout -k 10 300 python tools/shard_sim.py --config C2 | python -c "import sys,json; [print('units=$u', json.loads(l)['N'], json.loads(l)['tiles_ms'], json.loads(l)['tiles_chunks'], json.loads(l)['strata_ms']) for l in sys.stdin]"
done
