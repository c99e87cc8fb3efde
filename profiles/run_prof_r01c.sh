# Round 1, pass 3: parity suite, default bench line (C2 + CPU baseline), then per
# config (C2, C3, C4) a rocprofv3 kernel-trace/stats run and separate FETCH_SIZE /
# WRITE_SIZE PMC passes and a VALU/fp64 pass (no traces mixed with --pmc).
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${PASS:-r01c}
mkdir -p $O
cd $R
timeout -k 10 400 python -m pytest tests -q -m gpu -x > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python bench.py > $O/bench_default.log 2>&1
tail -1 $O/bench_default.log
for c in C2 C3 C4; do
  s=5; [ $c = C4 ] && s=2
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$c -o $c -- python bench.py --config $c --steps $s --warmup 1 --no-cpu-baseline > $O/trace_$c.log 2>&1
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_$c -o $c -- python bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline > $O/fetch_$c.log 2>&1
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write_$c -o $c -- python bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline > $O/write_$c.log 2>&1
  timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 GRBM_GUI_ACTIVE --output-format csv -d $O/valu_$c -o $c -- python bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline > $O/valu_$c.log 2>&1
  echo "$c profiled"
done
