# Run the GPU parity suite, then C2/C3/C4 single-GPU benches (no CPU baseline).
set -e
O=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 300 python -m pytest tests -q -m gpu -x > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for c in C2 C3 C4; do
  timeout -k 10 300 python bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_$c.log 2>&1
  python -c "import json,sys; d=json.loads(open('$O/bench_$c.log').read().strip().splitlines()[-1]); print('$c', d['value'], 'Msamples/s', d['ms_per_step'], 'ms/step', 'kernel', d['roofline']['kernel_ms'])"
done
