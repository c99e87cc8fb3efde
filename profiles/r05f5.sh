#!/bin/bash
# r05f5: the final tree -- default bench line and the default shard_sim (library units) for C2 at 1/2/4/8
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05f5
mkdir -p $O
timeout -k 10 600 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
timeout -k 10 600 python tools/shard_sim.py --config C2 > $O/shard_sim_C2.log 2>&1 || { tail $O/shard_sim_C2.log; exit 1; }
python -c "import json; d=json.loads(open('$O/bench_default.json').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['frac'], {c: v['value'] for c, v in d['other_configs'].items()})"
grep -h config $O/shard_sim_C2.log | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['N'], d['tiles_ms'], d['speedup_k'])"
