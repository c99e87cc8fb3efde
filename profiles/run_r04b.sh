#!/bin/bash
# r04b: A/B of the sign-selected node planes (build_dbgS0 = RT_SLAB_SIGN=0, the round-3 visit)
# on C3 and C5; of the C3 head unit size (RTX_HEAD_STRATA 64 / 128 / 256);
# and C4's noise cost (build_dbgN: turb() replaced by a constant -- same paths, no Perlin work)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04b
mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU_FMA_F32 GRBM_GUI_ACTIVE --output-format csv -d $O/ubench_pmc -o ub -- real-time-ray-tracing-engine_amd/build/ubench_issue > $O/ubench_pmc.log 2>&1 || { tail -20 $O/ubench_pmc.log; exit 1; }
bash profiles/ab.sh $O/slab_sign_ab.log "C3" "S0 base" 3 || exit 1
bash profiles/ab.sh $O/head_strata_ab.log "C3" "RTX_HEAD_STRATA=64 RTX_HEAD_STRATA=128 RTX_HEAD_STRATA=256" 2 || exit 1
bash profiles/ab.sh $O/noise_cost_ab.log "C4" "base N" 2 || exit 1
bash profiles/ab.sh $O/slab_sign_ab.log "C5" "S0 base" 1 || exit 1
for v in S0 base; do
  if [ $v = base ]; then L=$PWD/real-time-ray-tracing-engine_amd/build/librtx_hip.so; else L=$PWD/real-time-ray-tracing-engine_amd/build_dbg$v/librtx_hip.so; fi
  echo "== $v" >> $O/arity_sign_ab.log
  RTX_LIB=$L timeout -k 10 300 python tools/arity_ab.py --n 100000 1000000 --rounds 2 >> $O/arity_sign_ab.log 2>&1 || { tail -20 $O/arity_sign_ab.log; exit 1; }
done
tail -12 $O/arity_sign_ab.log
echo done
