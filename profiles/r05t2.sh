#!/bin/bash
# r05t2 (after tile order and the new tails): work-unit timelines (RT_UNIT_TIMES build, tools/unit_timeline.py): how
# much of a launch's span the wave slots spend without a unit -- C2 / C3 at
# one device and as an 8-way rank's share
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05t2
mkdir -p $O
export RTX_LIB=$PWD/real-time-ray-tracing-engine_amd/build_dbgT/librtx_hip.so
for args in "--config C2 --n 1" "--config C2 --n 8 --plan auto" "--config C2 --n 8 --plan chunks" "--config C2 --n 4 --plan auto" "--config C3 --n 1" "--config C3 --n 8 --plan auto"; do
  timeout -k 10 200 python tools/unit_timeline.py $args >> $O/timeline.log 2>> $O/timeline.err || { tail $O/timeline.err; exit 1; }
done
cat $O/timeline.log
