#!/bin/bash
# r05i: work-unit plans that write fewer chunk partials: C4 / C5
# as whole head tiles + a tail of finer chunks, vs the uniform split (rt_tuning via
# bench.py's RTX_TUNING); WRITE_SIZE of the render kernel for each plan
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05i
mkdir -p $O
bash profiles/ab.sh $O/c4_plan_ab.log "C4" "base RTX_TUNING=head_strata=1024,tail_tiles=1 RTX_TUNING=head_strata=1024,tail_tiles=1,tail_split=16 RTX_TUNING=head_strata=512" 2 || exit 1
bash profiles/ab.sh $O/c5_plan_ab.log "C5" "base RTX_TUNING=head_strata=4096,tail_tiles=1" 1 || exit 1
for v in base "head_strata=1024,tail_tiles=1" "head_strata=512"; do
  n=$(echo $v | tr ',=' '__')
  if [ "$v" = base ]; then unset RTX_TUNING; else export RTX_TUNING=$v; fi
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w_$n -o C4 -- python bench.py --config C4 --steps 1 --warmup 0 --no-cpu-baseline --no-other-configs --pmc off > $O/w_$n.log 2>&1 || { tail -20 $O/w_$n.log; exit 1; }
done
unset RTX_TUNING
echo done
