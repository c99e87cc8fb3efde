#!/bin/bash
# r04o: LDS and stall counters of the C3 render kernel on the DNodeL build (compare r04k, 64-B
# staged nodes)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04o
mkdir -p $O
B="python bench.py --config C3 --steps 1 --warmup 0 --no-cpu-baseline --no-other-configs --pmc off"
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d $O/a -o C3 -- $B > $O/a.log 2>&1 || { tail -20 $O/a.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $O/b -o C3 -- $B > $O/b.log 2>&1 || { tail -20 $O/b.log; exit 1; }
echo done
