# GPU parity suite + C2/C3/C4 bench lines (no CPU baseline); stops at the first failure.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
timeout -k 10 400 python -m pytest tests -q -m gpu -x > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for c in C2 C3 C4; do
  s=3; [ $c = C4 ] && s=2
  timeout -k 10 300 python bench.py --config $c --steps $s --warmup 1 --no-cpu-baseline > $O/bench_$c.log 2>&1
  python -c "import json; d=json.loads(open('$O/bench_$c.log').read().strip().splitlines()[-1]); print('$c', d['value'], 'Msamples/s kernel_ms', d['roofline']['kernel_ms'], 'frac', d['roofline']['frac'])"
done
