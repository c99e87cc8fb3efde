#!/bin/bash
# r04g: C3 A/B of the r04b build (build_dbgB) against the current one; C3 STATS line (two-walk
# model); 4-wide / binary arity A/B of the final visit forms against build_dbgS0; per-rank
# shard times (tools/shard_sim.py) C2-C5
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04g
mkdir -p $O
bash profiles/ab.sh $O/c3_build_ab.log "C3" "B base" 3 || exit 1
timeout -k 10 300 python bench.py --config C3 --steps 3 --warmup 1 --no-cpu-baseline --no-other-configs --pmc off > $O/bench_C3_stats.json 2> $O/bench_C3_stats.err || { tail -20 $O/bench_C3_stats.err; exit 1; }
for v in S0 base; do
  if [ $v = base ]; then L=$PWD/real-time-ray-tracing-engine_amd/build/librtx_hip.so; else L=$PWD/real-time-ray-tracing-engine_amd/build_dbg$v/librtx_hip.so; fi
  echo "== $v" >> $O/arity_sign_ab.log
  RTX_LIB=$L timeout -k 10 300 python tools/arity_ab.py --n 100000 1000000 --rounds 2 >> $O/arity_sign_ab.log 2>&1 || { tail -20 $O/arity_sign_ab.log; exit 1; }
done
grep -v amdgpu.ids $O/arity_sign_ab.log
for c in C2 C3 C4; do
  timeout -k 10 300 python tools/shard_sim.py --config $c > $O/shard_sim_$c.log 2>&1 || { tail -20 $O/shard_sim_$c.log; exit 1; }
  tail -1 $O/shard_sim_$c.log | cut -c1-200
done
timeout -k 10 400 python tools/shard_sim.py --config C5 --reps 2 > $O/shard_sim_C5.log 2>&1 || { tail -20 $O/shard_sim_C5.log; exit 1; }
tail -1 $O/shard_sim_C5.log | cut -c1-200
echo done
