# Round 2, pass e: instruction mix and stall counters of the C2 / C3 / C4 render
# kernels (current build), one rocprofv3 --pmc pass per counter group.
set -e
export TMPDIR=/tmp
O=gpurun_out/r02e
mkdir -p $O
for c in C2 C3 C4; do
  s=2; [ $c = C4 ] && s=1
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAVES --output-format csv -d $O/mix_$c -o mix -- python bench.py --config $c --steps $s --warmup 1 --no-cpu-baseline --pmc off --no-other-configs > $O/mix_$c.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d $O/stall_$c -o stall -- python bench.py --config $c --steps $s --warmup 1 --no-cpu-baseline --pmc off --no-other-configs > $O/stall_$c.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_FMA_F32 --output-format csv -d $O/f64_$c -o f64 -- python bench.py --config $c --steps $s --warmup 1 --no-cpu-baseline --pmc off --no-other-configs > $O/f64_$c.log 2>&1
  echo "$c done"
done
python - <<'PY'
import csv, glob, json
out = {}
for c in ("C2", "C3", "C4"):
    vals = {}
    for f in glob.glob("gpurun_out/r02e/*_%s/**/*counter_collection.csv" % c, recursive=True):
        for r in csv.DictReader(open(f)):
            if "render_tiles<false" in r["Kernel_Name"]:
                vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    out[c] = {k: sum(v) / len(v) for k, v in vals.items()}
json.dump(out, open("gpurun_out/r02e/summary.json", "w"), indent=1)
print(json.dumps({c: {k: "%.3g" % v for k, v in d.items()} for c, d in out.items()}, indent=1))
PY
