set -o pipefail
mkdir -p gpurun_out/r05f
L=real-time-ray-tracing-engine_amd
for v in base A B E; do
  if [ $v = base ]; then lib=$PWD/$L/build/librtx_hip.so; else lib=$PWD/$L/build_dbg$v/librtx_hip.so; fi
  RTX_LIB=$lib timeout -k 10 120 python tools/frame_dump.py --config C4 --spp 64 --out gpurun_out/r05f/c4_$v.npy > /dev/null || exit 1
done
for v in A B E; do python tools/frame_dump.py --compare gpurun_out/r05f/c4_base.npy gpurun_out/r05f/c4_$v.npy | sed "s/^/$v vs base: /"; done | tee gpurun_out/r05f/bitcmp.log
rm -f gpurun_out/r05f/*.npy
bash profiles/ab.sh gpurun_out/r05f/c4_rcp_ab.log "C4" "base E" 3 || exit 1
