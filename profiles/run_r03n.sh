#!/bin/bash
# r03n: the fog scene's Perlin table staged in LDS by the noise instances
# (base) vs read from HBM by the same build (RTX_LDS_PERLIN=0) vs the previous
# product (PL0: HBM table, octave loop unrolled).  Noise-instance parity, then
# C4 A/B; then the one-GPU shard simulation (tools/shard_sim.py) for C2/C3.
set -o pipefail
O=gpurun_out/r03n
mkdir -p $O
export PYTHONPATH=$PWD/real-time-ray-tracing-engine_amd:$PWD/tests:$PWD
timeout -k 10 400 python -u -m pytest tests/test_lds_perlin.py tests/test_gpu_instances.py tests/test_gpu_parity.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
bash profiles/ab.sh $O/ab.log "C4" "base RTX_LDS_PERLIN=0 PL0" 3 || exit 1
for c in C2 C3; do
  timeout -k 10 240 python -u tools/shard_sim.py --config $c > $O/shard_sim_$c.log 2>&1 || { tail -20 $O/shard_sim_$c.log; exit 1; }
  cat $O/shard_sim_$c.log
done
echo done
