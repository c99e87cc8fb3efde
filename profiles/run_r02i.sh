# Round 2, pass i: camera re-read from the kernarg segment at refills (base)
# vs the struct argument without re-read (K0) vs the previous build (Q0: separate
# arguments, full quad formulas); parity of base first.
set -e
O=gpurun_out/r02i
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_instances.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
bash profiles/ab_variants.sh base K0 Q0 base K0 2>&1 | tee $O/ab.log
