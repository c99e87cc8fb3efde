#!/bin/bash
# r05z6: two frames in flight in bench.py (--pipeline 2: consecutive frames on
# two streams with a scene each) vs one (--pipeline 1) -- C2 / C3 / C4, the
# bench-contract rehearsals (gloo 2 ranks, RCCL world of one), the default line
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05z6
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_bench_contract.py > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
for r in 1 2; do for c in C2 C3 C4; do
  case $c in C2) st=10;; C3) st=4;; C4) st=2;; esac
  for p in 2 1; do
    timeout -k 10 300 python bench.py --config $c --steps $st --warmup 2 --pipeline $p --no-cpu-baseline --pmc off --no-other-configs 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('pipe$p', '$c', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], flush=True)" || exit 1
  done
done; done | tee $O/ab.log
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --config C2 --steps 20 --warmup 2 --pg-rehearsal --check --no-cpu-baseline --pmc off --no-other-configs > $O/reh.json 2> $O/reh.err || { tail $O/reh.err; exit 1; }
python -c "import json; d=json.loads(open('$O/reh.json').read().strip().splitlines()[-1]); print('rehearsal', d['value'], d['ms_per_step'], d.get('check'), d['config']['parallelism'])"
