set -e
mkdir -p gpurun_out
bash profiles/ab_variants.sh base P5
export TMPDIR=/tmp
O=gpurun_out/pmc_c2
mkdir -p $O
B="python bench.py --config C2 --steps 1 --warmup 0 --no-cpu-baseline"
timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES --output-format csv -d $O/a -o C2 -- $B > $O/a.log 2>&1
timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv -d $O/c -o C2 -- $B > $O/c.log 2>&1
python tools/pmc_table.py $O/a/*/C2_counter_collection.csv $O/c/*/C2_counter_collection.csv 2>/dev/null || find $O -name "*.csv"
