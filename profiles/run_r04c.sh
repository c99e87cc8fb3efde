#!/bin/bash
# r04c: full GPU suite (new roofline test, C3 head plan of 128-strata chunks), smoke, the default
# bench line (new VALU figures), and the binary / 4-wide A/B of the shared sign-picked plane loads
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04c
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
timeout -k 10 600 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
tail -1 $O/bench_default.json | cut -c1-300
timeout -k 10 300 python bench.py --config C4 --steps 1 --warmup 1 --no-cpu-baseline --no-other-configs --pmc off > $O/bench_C4_stats.json 2> $O/bench_C4_stats.err || { tail -20 $O/bench_C4_stats.err; exit 1; }
for v in S0 base; do
  if [ $v = base ]; then L=$PWD/real-time-ray-tracing-engine_amd/build/librtx_hip.so; else L=$PWD/real-time-ray-tracing-engine_amd/build_dbg$v/librtx_hip.so; fi
  echo "== $v" >> $O/arity_sign_ab.log
  RTX_LIB=$L timeout -k 10 300 python tools/arity_ab.py --n 100000 1000000 --rounds 2 >> $O/arity_sign_ab.log 2>&1 || { tail -20 $O/arity_sign_ab.log; exit 1; }
done
cat $O/arity_sign_ab.log | grep -v amdgpu.ids
echo done
