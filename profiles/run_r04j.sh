#!/bin/bash
# r04j: C3 A/B -- the sphere-item leaf test (base: item i is sphere i, no item record read) against
# build_dbgSI0 (RT_SPHERE_ITEMS=0, the item record first), and two parked leaves per lane
# (RT_PARK2=1: build_dbgP2; =2, one leaf per lane per leaf phase: build_dbgP3; both without the
# sphere-item test); the base's C3 STATS line and the parity tests that cover the walk
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04j
mkdir -p $O
bash profiles/ab.sh $O/c3_ab.log "C3" "base SI0 P3 P2" 3 || exit 1
timeout -k 10 300 python bench.py --config C3 --steps 3 --warmup 1 --no-cpu-baseline --no-other-configs --pmc off > $O/bench_C3_stats.json 2> $O/bench_C3_stats.err || { tail -20 $O/bench_C3_stats.err; exit 1; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_persistent.py tests/test_c5.py tests/test_bvh4.py tests/test_device_bvh.py > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
echo done
