# Round 2, pass g: phase-cycle shares (STATS instance, s_memtime) and lane
# utilisation per config.
set -e
O=gpurun_out/r02g
mkdir -p $O
for c in C2 C3 C4; do
  timeout -k 10 200 python bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline --pmc off --no-other-configs > $O/$c.log 2>&1
  python -c "import json; d=json.loads(open('$O/$c.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$c', d['value'], r['lane_utilisation'], r.get('phase_share'))"
done
