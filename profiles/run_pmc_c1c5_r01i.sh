# PMC passes (FETCH_SIZE, WRITE_SIZE, VALU/fp64; one pass each, no traces) and a
# kernel-trace/stats run for configs C1 and C5, which had no traffic figure yet.
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r01i_pmc
mkdir -p $O
cd $R
for c in C1 C5; do
  s=3; w=1; [ $c = C5 ] && s=1 && w=0
  B="python bench.py --config $c --steps $s --warmup $w --no-cpu-baseline"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$c -o $c -- $B > $O/trace_$c.log 2>&1
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_$c -o $c -- $B > $O/fetch_$c.log 2>&1
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write_$c -o $c -- $B > $O/write_$c.log 2>&1
  timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 GRBM_GUI_ACTIVE --output-format csv -d $O/valu_$c -o $c -- $B > $O/valu_$c.log 2>&1
  echo "$c profiled"
done
