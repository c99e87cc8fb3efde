#!/bin/bash
# r06zz: final profile set of round 6 (probe-ordered build) -- full GPU suite, smoke, the driver's default line,
# per-config lines with their PMC summaries (bench.py --pmc-save: VALU / FETCH_SIZE /
# WRITE_SIZE passes), rocprofv3 --kernel-trace --stats of the driver's command (C2) and
# of C3 / C4 with steady-state summaries (tools/kernel_stats.py), and bench.py starting
# its own 2 ranks on this one GPU (gloo, --share-device, --check); the 8-way prediction
# (tools/shard_sim.py) for C2 and C3
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06zz
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
tail -1 $O/bench_default.json | cut -c1-200
for c in C4 C5; do
  timeout -k 10 400 python bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline --no-other-configs --pmc-save $O/pmc_$c.json > $O/bench_$c.json 2> $O/bench_$c.err || { tail -20 $O/bench_$c.err; exit 1; }
done
for c in C2 C3; do
  timeout -k 10 300 python bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-other-configs --pmc-save $O/pmc_$c.json > $O/bench_$c.json 2> $O/bench_$c.err || { tail -20 $O/bench_$c.err; exit 1; }
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_C2 -o C2 -- python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-other-configs --pmc off > $O/trace_C2.json 2> $O/trace_C2.err || { tail -20 $O/trace_C2.err; exit 1; }
for c in C3 C4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$c -o $c -- python bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline --no-other-configs --pmc off > $O/trace_$c.json 2> $O/trace_$c.err || { tail -20 $O/trace_$c.err; exit 1; }
done
python tools/kernel_stats.py $(find $O/trace_C2 -name "*kernel_trace.csv") --skip 5 --steps 20 --out $O/C2_kernel_stats_steady.csv 2>&1 | tee $O/steady.log
for c in C3 C4; do
  python tools/kernel_stats.py $(find $O/trace_$c -name "*kernel_trace.csv") --skip 1 --steps 5 --out $O/${c}_kernel_stats_steady.csv 2>&1 | tee -a $O/steady.log
done
find $O -name "*kernel_trace.csv" -delete
timeout -k 10 300 python bench.py --gpus 2 --backend gloo --share-device --config C2 --steps 5 --warmup 1 --check > $O/launcher_2rank_C2.json 2> $O/launcher_2rank_C2.err || { tail -20 $O/launcher_2rank_C2.err; exit 1; }
tail -1 $O/launcher_2rank_C2.json | cut -c1-200
for c in C2 C3; do
  timeout -k 10 300 python tools/shard_sim.py --config $c > $O/shard_sim_$c.log 2>&1 || { tail -20 $O/shard_sim_$c.log; exit 1; }
  tail -4 $O/shard_sim_$c.log
done
echo done
