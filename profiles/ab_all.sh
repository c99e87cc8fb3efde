# GPU parity suite with base, then C2/C3/C4 A/B of library variants (build_dbg<V>; "base" = build/)
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
for v in "$@"; do
  case $v in
    base) L=$PWD/real-time-ray-tracing-engine_amd/build/librtx_hip.so ;;
    *) L=$PWD/real-time-ray-tracing-engine_amd/build_dbg$v/librtx_hip.so ;;
  esac
  if [ "$v" != base ]; then RTX_LIB=$L timeout -k 10 300 python -u -m pytest tests/test_gpu_instances.py tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread 2>&1 | tail -1; fi
  for c in C2 C3 C4; do
    s=5; [ $c = C4 ] && s=2
    RTX_LIB=$L timeout -k 10 200 python bench.py --config $c --steps $s --warmup 1 --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$v', '$c', d['value'])"
  done
done
