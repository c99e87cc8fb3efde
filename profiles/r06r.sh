#!/bin/bash
# r06r: C4 work-unit plans with fewer chunk partials on the round-6 build (rt_tuning via
# RTX_TUNING): whole-tile heads with a tail of half / one tile per wave slot, 512-strata
# heads -- rate, and WRITE_SIZE of the render kernel per plan
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06r
mkdir -p $O
bash profiles/ab.sh $O/ab_C4.log "C4" "base RTX_TUNING=head_strata=1024,tail_tiles=0.5 RTX_TUNING=head_strata=1024,tail_tiles=1 RTX_TUNING=head_strata=512" 2 || exit 1
for v in base "head_strata=1024,tail_tiles=0.5"; do
  n=$(echo $v | tr ',=' '__')
  if [ "$v" = base ]; then unset RTX_TUNING; else export RTX_TUNING=$v; fi
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w_$n -o C4 -- python bench.py --config C4 --steps 1 --warmup 0 --no-cpu-baseline --no-other-configs --pmc off > $O/w_$n.log 2>&1 || { tail -20 $O/w_$n.log; exit 1; }
done
unset RTX_TUNING
python - <<'PY'
import csv, glob
for d in sorted(glob.glob("gpurun_out/r06r/w_*")):
    if not d.endswith(".log"):
        for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                if "render_tiles<false" in r["Kernel_Name"]:
                    print(d, r["Counter_Name"], float(r["Counter_Value"]) * 1024 / 1e6, "MB")
PY
echo done
