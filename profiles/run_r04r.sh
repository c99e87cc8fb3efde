#!/bin/bash
# r04r: noise albedos deferred to the end of the path trip and evaluated with the octaves spread
# over the wave (base, RT_NOISE_WAVE=1) against inline evaluation (build_dbgNW0): the C4 frame
# bit for bit (full size), C4 A/B x3, the C4 STATS line, the noise parity tests
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04r
mkdir -p $O
L0=$PWD/real-time-ray-tracing-engine_amd/build_dbgNW0/librtx_hip.so
timeout -k 10 200 python tools/frame_dump.py --config C4 --out $O/c4_base.npy > $O/dump.log 2>&1 || { tail -20 $O/dump.log; exit 1; }
RTX_LIB=$L0 timeout -k 10 200 python tools/frame_dump.py --config C4 --out $O/c4_nw0.npy >> $O/dump.log 2>&1 || { tail -20 $O/dump.log; exit 1; }
python tools/frame_dump.py --compare $O/c4_base.npy $O/c4_nw0.npy | tee $O/bitcmp.log
rm -f $O/*.npy
timeout -k 10 600 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_lds_perlin.py tests/test_statistical_parity.py > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
bash profiles/ab.sh $O/c4_ab.log "C4" "base NW0" 3 || exit 1
timeout -k 10 300 python bench.py --config C4 --steps 1 --warmup 1 --no-cpu-baseline --no-other-configs --pmc off > $O/bench_C4_stats.json 2> $O/bench_C4_stats.err || { tail -20 $O/bench_C4_stats.err; exit 1; }
echo done
