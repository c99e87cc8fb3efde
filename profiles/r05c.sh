set -o pipefail
mkdir -p gpurun_out/r05c
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_instances.py tests/test_medium_box.py > gpurun_out/r05c/gpu_tests.log 2>&1 || { tail -30 gpurun_out/r05c/gpu_tests.log; exit 1; }
tail -2 gpurun_out/r05c/gpu_tests.log
bash profiles/ab.sh gpurun_out/r05c/c4_ab.log "C4" "base B" 3 || exit 1
