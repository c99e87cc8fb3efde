# Round 1 pass 2: GPU parity suite, default bench (C2 + CPU baseline), C3/C4
# lines, rocprofv3 kernel trace + separate FETCH_SIZE / WRITE_SIZE passes on C2.
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O/prof
cd $R
timeout -k 10 400 python -m pytest tests -q -m gpu -x > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python bench.py > $O/bench_default.log 2>&1
tail -1 $O/bench_default.log
for c in C3 C4; do
  timeout -k 10 300 python bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_$c.log 2>&1
  tail -1 $O/bench_$c.log
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof/trace -o c2 -- python bench.py --config C2 --steps 5 --warmup 1 --no-cpu-baseline > $O/prof_trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/prof/pmc_fetch -o c2 -- python bench.py --config C2 --steps 2 --warmup 1 --no-cpu-baseline > $O/prof_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/prof/pmc_write -o c2 -- python bench.py --config C2 --steps 2 --warmup 1 --no-cpu-baseline > $O/prof_write.log 2>&1
echo done
