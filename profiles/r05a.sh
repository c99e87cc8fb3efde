set -o pipefail
mkdir -p gpurun_out/r05a
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_medium_box.py tests/test_gpu_parity.py tests/test_cli.py tests/test_bvh4.py tests/test_multi.py tests/test_dist.py > gpurun_out/r05a/gpu_tests.log 2>&1 || { tail -30 gpurun_out/r05a/gpu_tests.log; exit 1; }
tail -3 gpurun_out/r05a/gpu_tests.log
timeout -k 10 200 python bench.py --config C4 --steps 2 --warmup 1 --no-cpu-baseline --pmc off --no-other-configs > gpurun_out/r05a/bench_C4.json 2> gpurun_out/r05a/bench_C4.err || exit 1
bash profiles/ab.sh gpurun_out/r05a/c4_ab.log "C4" "base A" 3 || exit 1
