# GPU parity tests, SIMD-efficiency counters and an A/B of library variants (C2/C3/C4).
# usage: bash profiles/ab_quick.sh V1 V2 ...   (variants under real-time-ray-tracing-engine_amd/build_dbg<V>; "base" = build/)
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
bash profiles/simd_stats.sh
bash profiles/ab_variants.sh "$@"
