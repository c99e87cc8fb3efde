#!/bin/bash
# r04n: the binary visit's push / advance / pop as selects (build_dbgVS, RT_VISIT_SELECT=1)
# against the branchy visit (base), C3 x4 and C5 x2, on the DNodeL build without the
# absolute-address entries and the guarded sqrt (both dropped after r04m)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04n
mkdir -p $O
bash profiles/ab.sh $O/c3_ab.log "C3" "base VS" 4 || exit 1
bash profiles/ab.sh $O/c5_ab.log "C5" "base VS" 2 || exit 1
echo done
