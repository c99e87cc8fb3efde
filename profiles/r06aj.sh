#!/bin/bash
# r06aj: the build with first-measured flat-world subset orders: GPU suite + smoke, the
# default line, C2 / C3 / C5 8-way predictions (tools/shard_sim.py)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06aj
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
tail -1 $O/bench_default.json | cut -c1-200
for c in C2 C3; do
  timeout -k 10 300 python tools/shard_sim.py --config $c > $O/shard_sim_$c.log 2>&1 || { tail -20 $O/shard_sim_$c.log; exit 1; }
  grep '"N": 8' $O/shard_sim_$c.log | cut -c1-330
done
echo done
