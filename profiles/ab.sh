#!/bin/bash
# A/B timing of library variants: ab.sh OUT "CONFIGS" "VARIANTS" REPS
#   variant "base" = real-time-ray-tracing-engine_amd/build, X = .../build_dbgX,
#   NAME=VALUE = the base library with that environment variable; interleaved reps
set -o pipefail
OUT=$1; CONFIGS=$2; VARIANTS=$3; REPS=${4:-2}
for r in $(seq $REPS); do
  for c in $CONFIGS; do
    case $c in C2) st=10;; C3) st=4;; C4) st=2;; C5) st=1;; *) st=3;; esac
    for v in $VARIANTS; do
      EV=""
      if [ $v = base ]; then L=$PWD/real-time-ray-tracing-engine_amd/build/librtx_hip.so;
      elif [[ $v == *=* ]]; then L=$PWD/real-time-ray-tracing-engine_amd/build/librtx_hip.so; EV=$v;
      else L=$PWD/real-time-ray-tracing-engine_amd/build_dbg$v/librtx_hip.so; fi
      env $EV RTX_LIB=$L timeout -k 10 200 python bench.py --config $c --steps $st --warmup 1 --no-cpu-baseline --pmc off --no-other-configs 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$v', '$c', d['value'], d['roofline']['kernel_ms'], flush=True)" || exit 1
    done
  done
done | tee -a $OUT
