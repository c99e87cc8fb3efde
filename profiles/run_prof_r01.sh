set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O/prof
cd $R
timeout -k 10 300 python bench.py --config C3 --steps 2 --warmup 1 --no-cpu-baseline > $O/bench_c3.log 2>&1
timeout -k 10 300 python bench.py --config C4 --steps 1 --warmup 1 --no-cpu-baseline > $O/bench_c4.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof/trace -o c2 -- python bench.py --config C2 --steps 5 --warmup 1 --no-cpu-baseline > $O/prof_trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/prof/pmc_fetch -o c2 -- python bench.py --config C2 --steps 2 --warmup 1 --no-cpu-baseline > $O/prof_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/prof/pmc_write -o c2 -- python bench.py --config C2 --steps 2 --warmup 1 --no-cpu-baseline > $O/prof_write.log 2>&1
echo done
