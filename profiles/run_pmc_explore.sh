# PMC exploration on the render kernel: instruction mix, stall breakdown, f64 op mix.
# Each pass is its own rocprofv3 run (SQ has 8 slots per pass); --pmc only, no traces.
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
CFG=${1:-C3}
mkdir -p $O/pmc
cd $R
rocprofv3 -L > $O/pmc/counters_list.txt 2>&1 || true
B="python bench.py --config $CFG --steps 1 --warmup 0 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH --output-format csv -d $O/pmc/a -o $CFG -- $B > $O/pmc/a.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d $O/pmc/b -o $CFG -- $B > $O/pmc/b.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_MISC --output-format csv -d $O/pmc/c -o $CFG -- $B > $O/pmc/c.log 2>&1
echo done
