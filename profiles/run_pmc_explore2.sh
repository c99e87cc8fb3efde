# PMC: stall breakdown + cache behaviour of the render kernel for one config.
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
CFG=${1:-C3}
O=$R/gpurun_out/pmc2_$CFG
mkdir -p $O
cd $R
B="python bench.py --config $CFG --steps 1 --warmup 0 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES --output-format csv -d $O/a -o $CFG -- $B > $O/a.log 2>&1
timeout -k 10 300 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --output-format csv -d $O/b -o $CFG -- $B > $O/b.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_INST_LEVEL_VMEM SQ_LEVEL_WAVES --output-format csv -d $O/c -o $CFG -- $B > $O/c.log 2>&1
echo done
