#!/bin/bash
# r04k: the gfx950 counter list, and a stall / LDS breakdown of the C3 render kernel (two PMC
# passes of one C3 frame each)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04k
mkdir -p $O
timeout -k 10 120 rocprofv3 -L > $O/counters_all.txt 2>&1 || { tail -5 $O/counters_all.txt; exit 1; }
B="python bench.py --config C3 --steps 1 --warmup 0 --no-cpu-baseline --no-other-configs --pmc off"
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d $O/a -o C3 -- $B > $O/a.log 2>&1 || { tail -20 $O/a.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $O/b -o C3 -- $B > $O/b.log 2>&1 || { tail -20 $O/b.log; exit 1; }
find $O -name "*counter_collection.csv"
echo done
