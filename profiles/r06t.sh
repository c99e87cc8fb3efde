#!/bin/bash
# r06t: C4 whole-tile heads under the probe's order (build_dbgN), tail size x split
# chosen so the chunk partials stay <= 0.5x the frame, vs the default plan; WRITE_SIZE
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06t
mkdir -p $O
N=$PWD/real-time-ray-tracing-engine_amd/build_dbgN/librtx_hip.so
run() { # label tuning
  RTX_LIB=$N RTX_TUNING=$2 timeout -k 10 200 python bench.py --config C4 --steps 2 --warmup 1 --no-cpu-baseline --pmc off --no-other-configs 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$1', 'C4', d['value'], d['roofline']['kernel_ms'], flush=True)"
}
for r in 1 2 3; do
  run N "" || exit 1
  run N_t1_s8 "head_strata=1024,tail_tiles=1" || exit 1
  run N_t1_s4 "head_strata=1024,tail_tiles=1,tail_split=4" || exit 1
  run N_t2_s2 "head_strata=1024,tail_tiles=2,tail_split=2" || exit 1
  run N_t0.5_s8 "head_strata=1024,tail_tiles=0.5" || exit 1
done 2>&1 | tee $O/ab_C4.log
for v in "head_strata=1024,tail_tiles=1,tail_split=4" "head_strata=1024,tail_tiles=2,tail_split=2" "head_strata=1024,tail_tiles=0.5"; do
  n=$(echo $v | tr ',=' '__')
  RTX_LIB=$N RTX_TUNING=$v timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w_$n -o C4 -- python bench.py --config C4 --steps 1 --warmup 0 --no-cpu-baseline --no-other-configs --pmc off > $O/w_$n.log 2>&1 || { tail -20 $O/w_$n.log; exit 1; }
done
python - <<'PY' | tee $O/write_size.log
import csv, glob
for d in sorted(glob.glob("gpurun_out/r06t/w_*")):
    if not d.endswith(".log"):
        for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                if "render_tiles<false" in r["Kernel_Name"]:
                    print(d, r["Counter_Name"], float(r["Counter_Value"]) * 1024 / 1e6, "MB")
PY
echo done
