# Round 2, pass c: parity of the resumable-walk kernel (default build), then an
# A/B of RT_RESUME=0 and RT_SHADE_MIN variants on C2/C3/C4, and the C3 lane
# utilisation of the default build.
set -e
export TMPDIR=/tmp
O=gpurun_out/r02c
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_instances.py tests/test_statistical_parity.py tests/test_multi.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
bash profiles/ab_variants.sh base R0 S8 S16 S48 2>&1 | tee $O/ab.log
timeout -k 10 200 python bench.py --config C3 --steps 3 --warmup 1 --no-cpu-baseline --pmc off > $O/c3.log 2>&1
python -c "import json; d=json.loads(open('$O/c3.log').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['lane_utilisation'])"
