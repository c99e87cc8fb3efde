#!/bin/bash
# r03q: merged regeneration with the camera frame read afresh for the new rays (MC) vs the old trip (M0) vs merged (base)
set -o pipefail
O=gpurun_out/r03q
mkdir -p $O
export PYTHONPATH=$PWD/real-time-ray-tracing-engine_amd:$PWD/tests:$PWD
true
tail -1 $O/gpu_tests.log
bash profiles/ab.sh $O/ab.log "C2" "MC M0 base" 3 || exit 1
echo done
