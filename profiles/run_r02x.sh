# Round 2, pass x (run with PASS=r02x; final build after merged shading): GPU parity suite (incl. rt_multi / CLI shards / live-PMC bench
# line), default bench line (live PMC passes + reference -p CPU baseline), then a
# kernel-trace/stats run of the same C2 command.
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${PASS:-r02b}
mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 420 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
timeout -k 10 400 python bench.py > $O/bench_default.log 2> $O/bench_default.err
tail -1 $O/bench_default.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_C2 -o C2 -- python bench.py --config C2 --steps 5 --warmup 1 --no-cpu-baseline --pmc off > $O/trace_C2.log 2>&1
tail -1 $O/trace_C2.log
