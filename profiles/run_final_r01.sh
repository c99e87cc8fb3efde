# Round-end rehearsal: GPU parity suite, smoke(), default bench (with CPU baseline); stops at the first failure.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -v -m gpu -x --timeout 120 --timeout-method thread > $O/final_gpu_tests.log 2>&1 || { tail -40 $O/final_gpu_tests.log; exit 1; }
tail -1 $O/final_gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/final_smoke.log 2>&1 || { tail -20 $O/final_smoke.log; exit 1; }
tail -1 $O/final_smoke.log
timeout -k 10 300 python bench.py > $O/final_bench_default.log 2>&1 || { tail -20 $O/final_bench_default.log; exit 1; }
tail -1 $O/final_bench_default.log
