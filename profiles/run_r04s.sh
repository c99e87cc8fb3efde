#!/bin/bash
# r04s: instruction-cache and issue counters of the render kernel: C4 with and without the
# wave-spread noise octaves (base / build_dbgNW0), C2 and C3 (base)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04s
mkdir -p $O
CTR="SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
for v in base NW0; do
  L=$PWD/real-time-ray-tracing-engine_amd/build/librtx_hip.so
  [ $v = NW0 ] && L=$PWD/real-time-ray-tracing-engine_amd/build_dbgNW0/librtx_hip.so
  RTX_LIB=$L timeout -s KILL 300 rocprofv3 --pmc $CTR --output-format csv -d $O/C4_$v -o C4 -- python bench.py --config C4 --steps 1 --warmup 0 --no-cpu-baseline --no-other-configs --pmc off > $O/C4_$v.log 2>&1 || { tail -20 $O/C4_$v.log; exit 1; }
done
for c in C2 C3; do
  timeout -s KILL 300 rocprofv3 --pmc $CTR --output-format csv -d $O/$c -o $c -- python bench.py --config $c --steps 1 --warmup 0 --no-cpu-baseline --no-other-configs --pmc off > $O/$c.log 2>&1 || { tail -20 $O/$c.log; exit 1; }
done
echo done
