# A/B: LDS-staged BVH prefix (default budget) vs none, and a few fixed budgets.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out
for c in C3 C4 C2; do
  for n in default 0 64 512; do
    if [ $n = default ]; then unset RTX_LDS_NODES; else export RTX_LDS_NODES=$n; fi
    s=3; [ $c = C4 ] && s=1
    timeout -k 10 200 python bench.py --config $c --steps $s --warmup 1 --no-cpu-baseline > $O/ab_$c_$n.log 2>&1
    python -c "import json; d=json.loads(open('$O/ab_$c_$n.log').read().strip().splitlines()[-1]); print('$c lds_nodes=$n', d['value'], d['roofline']['kernel_ms'])"
  done
done
unset RTX_LDS_NODES
