#!/bin/bash
# r05l: sphere-light cone terms shared by light sampling and the light pdf
# (base) vs computed at both sites (G, RT_LIGHT_CONE=0): bit-compare + A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05l
mkdir -p $O
L=real-time-ray-tracing-engine_amd
for c in C2 C4; do
  for v in base G; do
    if [ $v = base ]; then lib=$PWD/$L/build/librtx_hip.so; else lib=$PWD/$L/build_dbg$v/librtx_hip.so; fi
    RTX_LIB=$lib timeout -k 10 120 python tools/frame_dump.py --config $c --spp 64 --out $O/${c}_$v.npy > /dev/null || exit 1
  done
  python tools/frame_dump.py --compare $O/${c}_base.npy $O/${c}_G.npy | sed "s/^/$c cone G vs base: /" | tee -a $O/bitcmp.log
done
rm -f $O/*.npy
bash profiles/ab.sh $O/ab.log "C4 C2" "base G" 3 || exit 1
echo done
