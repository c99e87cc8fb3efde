#!/bin/bash
# r05q: the data movement of an in-block trace / shade role split, measured
# without the split (RT_XCHG_PROBE=1, build_dbgX): frames bit-compared, C2 / C4 A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05q
mkdir -p $O
L=real-time-ray-tracing-engine_amd
for c in C2 C4; do
  for v in base X; do
    if [ $v = base ]; then lib=$PWD/$L/build/librtx_hip.so; else lib=$PWD/$L/build_dbg$v/librtx_hip.so; fi
    RTX_LIB=$lib timeout -k 10 120 python tools/frame_dump.py --config $c --spp 64 --out $O/${c}_$v.npy > /dev/null || exit 1
  done
  python tools/frame_dump.py --compare $O/${c}_base.npy $O/${c}_X.npy | sed "s/^/$c probe X vs base: /" | tee -a $O/bitcmp.log
done
rm -f $O/*.npy
bash profiles/ab.sh $O/ab.log "C2 C4" "base X" 2 || exit 1
echo done
