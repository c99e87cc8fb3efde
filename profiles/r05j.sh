#!/bin/bash
# r05j: where C3's LDS bank conflicts come from -- counter experiments (results
# not used): the pixel accumulator's ds_add_f64 made lane-private (Q build),
# the world items and spheres left in HBM (no_lds_prims); plus the r05i plan sweep
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05j
mkdir -p $O
L=real-time-ray-tracing-engine_amd
B="python bench.py --config C3 --steps 1 --warmup 0 --no-cpu-baseline --no-other-configs --pmc off"
run() { # name lib tuning
  RTX_LIB=$2 RTX_TUNING=$3 timeout -s KILL 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_$1 -o C3 -- $B > $O/pmc_$1.log 2>&1 || { tail -20 $O/pmc_$1.log; exit 1; }
}
run base $PWD/$L/build/librtx_hip.so "" || exit 1
run acc_lane $PWD/$L/build_dbgQ/librtx_hip.so "" || exit 1
run no_prims $PWD/$L/build/librtx_hip.so "no_lds_prims=1" || exit 1
bash profiles/r05i.sh || exit 1
echo done
