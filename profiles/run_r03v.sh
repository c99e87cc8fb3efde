#!/bin/bash
# r03v: sincos polynomial constants materialised at their use (two s_mov_b32 + one
# v_fma_f64 with the SGPR pair, instead of 10 hoisted VGPR pairs and v_mov_b64 + v_fmac_f64
# per step): full GPU suite, then C2/C3/C4 A/B against the hoisted form (K0)
set -o pipefail
O=gpurun_out/r03v
mkdir -p $O
export PYTHONPATH=$PWD/real-time-ray-tracing-engine_amd:$PWD/tests:$PWD
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
bash profiles/ab.sh $O/ab.log "C2 C3 C4" "base K0" 2 || exit 1
echo done
