set -o pipefail
mkdir -p gpurun_out/r05g
L=real-time-ray-tracing-engine_amd
for v in base F; do
  if [ $v = base ]; then lib=$PWD/$L/build/librtx_hip.so; else lib=$PWD/$L/build_dbg$v/librtx_hip.so; fi
  RTX_LIB=$lib timeout -k 10 120 python tools/frame_dump.py --config C4 --spp 64 --out gpurun_out/r05g/c4_$v.npy > /dev/null || exit 1
done
python tools/frame_dump.py --compare gpurun_out/r05g/c4_base.npy gpurun_out/r05g/c4_F.npy | sed "s/^/F vs base: /" | tee gpurun_out/r05g/bitcmp.log
rm -f gpurun_out/r05g/*.npy
bash profiles/ab.sh gpurun_out/r05g/c4_sincos_ab.log "C4" "base F" 3 || exit 1
timeout -k 10 200 python tools/scene_rate.py --help > /dev/null 2>&1
