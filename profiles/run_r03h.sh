#!/bin/bash
# r03h: one-wave blocks for the flat instances, Perlin FMA/lerp form, traversal stack as a
# pointer without overflow guard, persistent instance also for tile-subset launches.
# Full GPU suite, then A/B: base vs B1 (r03g's one-wave build: old stack code, reference
# Perlin order) vs SG (base + stack overflow guard).
set -o pipefail
O=gpurun_out/r03h
mkdir -p $O
export PYTHONPATH=$PWD/real-time-ray-tracing-engine_amd:$PWD/tests:$PWD
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
bash profiles/ab.sh $O/ab.log "C3 C4 C2" "base B1 SG" 2 || exit 1
echo done
