#!/bin/bash
# r06v: C3 / C5 whole-tile heads (fewer chunk partials) now that the
# plain instances dispatch tiles most expensive first: rate and WRITE_SIZE (build_dbgM)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06v
mkdir -p $O
M=$PWD/real-time-ray-tracing-engine_amd/build_dbgM/librtx_hip.so
run() { # label config tuning steps
  RTX_LIB=$M RTX_TUNING=$3 timeout -k 10 300 python bench.py --config $2 --steps $4 --warmup 1 --no-cpu-baseline --pmc off --no-other-configs 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$1', '$2', d['value'], d['roofline']['kernel_ms'], flush=True)"
}
for r in 1 2; do
  run base C3 "" 4 || exit 1
  run h256 C3 "head_strata=256" 4 || exit 1
  run h256_t0.5 C3 "head_strata=256,tail_tiles=0.5" 4 || exit 1
done 2>&1 | tee $O/ab_C3.log
run base C5 "" 1 2>&1 | tee $O/ab_C5.log || exit 1
run h4096 C5 "head_strata=4096" 1 2>&1 | tee -a $O/ab_C5.log || exit 1
for spec in "C3 base" "C3 head_strata=256" "C5 base" "C5 head_strata=4096"; do
  set -- $spec
  t=$2; [ "$t" = base ] && t=""
  n=$(echo $1_$2 | tr ',=' '__')
  RTX_LIB=$M RTX_TUNING=$t timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w_$n -o $1 -- python bench.py --config $1 --steps 1 --warmup 0 --no-cpu-baseline --no-other-configs --pmc off > $O/w_$n.log 2>&1 || { tail -20 $O/w_$n.log; exit 1; }
done
python - <<'PY' | tee $O/write_size.log
import csv, glob
for d in sorted(glob.glob("gpurun_out/r06v/w_*")):
    if not d.endswith(".log"):
        for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
            v = [float(r["Counter_Value"]) for r in csv.DictReader(open(f)) if "render_tiles<false" in r["Kernel_Name"]]
            print(d, "WRITE_SIZE per launch", round(sum(v) / max(1, len(v)) * 1024 / 1e6, 1), "MB over", len(v), "launches")
PY
echo done
