# N=1 layout A/B: frame-direct vs tile work units (+chunk sum + reorder), with --check.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
for c in C2 C3 C4; do
  s=5; [ $c = C3 ] && s=3; [ $c = C4 ] && s=2
  for l in frame tiles; do
    timeout -k 10 300 python bench.py --config $c --steps $s --warmup 1 --no-cpu-baseline --check --n1-layout $l > $O/n1_${c}_$l.log 2>&1 || { tail -20 $O/n1_${c}_$l.log; exit 1; }
    python -c "import json; d=json.loads(open('$O/n1_${c}_$l.log').read().strip().splitlines()[-1]); print('$c $l', d['value'], 'ms', d['ms_per_step'], 'kernel', d['roofline']['kernel_ms'], d['check'])"
  done
done
