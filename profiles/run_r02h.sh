# Round 2, pass h: axis-aligned quad formulas -- parity (quad scenes) and A/B
# against the full formulas (RT_QUAD_AA=0) on C2/C3/C4.
set -e
O=gpurun_out/r02h
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_instances.py tests/test_statistical_parity.py tests/test_stored_form.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
bash profiles/ab_variants.sh base Q0 base Q0 2>&1 | tee $O/ab.log
