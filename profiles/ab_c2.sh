# C2-only A/B of library variants (libs under real-time-ray-tracing-engine_amd/build_dbg<V>; "base" = build/)
for v in "$@"; do
  if [ "$v" = base ]; then L=$PWD/real-time-ray-tracing-engine_amd/build/librtx_hip.so; else L=$PWD/real-time-ray-tracing-engine_amd/build_dbg$v/librtx_hip.so; fi
  RTX_LIB=$L timeout -k 10 200 python bench.py --config C2 --steps 10 --warmup 2 --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$v', 'C2', d['value'])"
done
