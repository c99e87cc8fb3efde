# usage: perf_variants.sh V1 V3 ... (libs under real-time-ray-tracing-engine_amd/build_dbg<V>); "base" = build/
for v in "$@"; do
  if [ "$v" = base ]; then L=$PWD/real-time-ray-tracing-engine_amd/build/librtx_hip.so; else L=$PWD/real-time-ray-tracing-engine_amd/build_dbg$v/librtx_hip.so; fi
  for c in C2 C3 C4; do
    s=3; [ $c = C4 ] && s=1
    RTX_LIB=$L timeout -k 10 200 python bench.py --config $c --steps $s --warmup 1 --no-cpu-baseline --pmc off --no-other-configs 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$v', '$c', d['value'])"
  done
done
