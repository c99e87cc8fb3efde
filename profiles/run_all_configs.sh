# One bench line per BASELINE config on one GPU (C5 with a single step).
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/allcfg
mkdir -p $O
for c in C1 C2 C3 C4 C5; do
  s=5; w=1
  [ $c = C4 ] && s=2
  [ $c = C5 ] && s=1 && w=0
  timeout -k 10 300 python bench.py --config $c --steps $s --warmup $w --no-cpu-baseline --check > $O/$c.log 2>&1
  python -c "import json; d=json.loads(open('$O/$c.log').read().strip().splitlines()[-1]); print('$c', d['config']['workload'], d['value'], 'Msamples/s', d['ms_per_step'], 'ms/step, frac', d['roofline']['frac'], d['check'])"
done
