set -o pipefail
mkdir -p gpurun_out/r05d
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_persistent.py tests/test_progressive.py tests/test_statistical_parity.py tests/test_stored_form.py tests/test_leaf_share.py tests/test_lds_perlin.py tests/test_multi.py tests/test_gpu_instances.py > gpurun_out/r05d/gpu_tests.log 2>&1 || { tail -30 gpurun_out/r05d/gpu_tests.log; exit 1; }
tail -2 gpurun_out/r05d/gpu_tests.log
