#!/bin/bash
# r03e: frame launches as whole-tile units with only the last tiles split into stratum chunks
# (tail split; split_sum_kernel over those tiles only) + scalar loads in the plain flat
# instance only.  Full GPU suite, then A/B of the tail size: RTX_TAIL_TILES = tiles split per
# wave slot (0 = every tile split, the round-2 rule).
set -o pipefail
O=gpurun_out/r03e
mkdir -p $O
export PYTHONPATH=$PWD/real-time-ray-tracing-engine_amd:$PWD/tests:$PWD
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
bash profiles/ab.sh $O/ab.log "C2 C3 C4" "base RTX_TAIL_TILES=0 RTX_TAIL_TILES=2 RTX_TAIL_TILES=0.5" 2 || exit 1

python bench.py --config C4 --steps 1 --warmup 0 --pmc off --no-cpu-baseline --no-other-configs 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=d['roofline']; print('C4 stats', json.dumps({k: r[k] for k in ('counters', 'phase_share', 'lane_utilisation')}))" | tee $O/c4_stats.log
echo done
