# A/B: frame-launch stratum chunking target (work units per resident wave); 0 = off.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out
for c in C2 C3 C4; do
  for t in 0 8 16 32; do
    export RTX_CHUNK_TARGET=$t
    s=3; [ $c = C4 ] && s=1
    timeout -k 10 200 python bench.py --config $c --steps $s --warmup 1 --no-cpu-baseline --check > $O/abc_$c_$t.log 2>&1
    python -c "import json; d=json.loads(open('$O/abc_$c_$t.log').read().strip().splitlines()[-1]); print('$c target=$t', d['value'], d['roofline']['kernel_ms'], d['check'])"
  done
done
unset RTX_CHUNK_TARGET
