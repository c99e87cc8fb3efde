#!/bin/bash
# r05h: 16-bit traversal stacks + 88-B DNodeL + 80-B LDS spheres in the persistent
# instance (base) vs the previous build (P); merged shading sincos (base) vs
# without (F); GPU tests of the touched paths; C3 LDS / stall counters for both
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05h
mkdir -p $O
L=real-time-ray-tracing-engine_amd
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_bvh4.py tests/test_lds_perlin.py > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
for v in base F; do
  if [ $v = base ]; then lib=$PWD/$L/build/librtx_hip.so; else lib=$PWD/$L/build_dbg$v/librtx_hip.so; fi
  RTX_LIB=$lib timeout -k 10 120 python tools/frame_dump.py --config C4 --spp 64 --out $O/c4_$v.npy > /dev/null || exit 1
done
python tools/frame_dump.py --compare $O/c4_base.npy $O/c4_F.npy | sed "s/^/C4 sincos F vs base: /" | tee $O/bitcmp.log
for v in base P; do
  if [ $v = base ]; then lib=$PWD/$L/build/librtx_hip.so; else lib=$PWD/$L/build_dbg$v/librtx_hip.so; fi
  RTX_LIB=$lib timeout -k 10 120 python tools/frame_dump.py --config C3 --spp 64 --out $O/c3_$v.npy > /dev/null || exit 1
done
python tools/frame_dump.py --compare $O/c3_base.npy $O/c3_P.npy | sed "s/^/C3 stack16 P vs base: /" | tee -a $O/bitcmp.log
rm -f $O/*.npy
bash profiles/ab.sh $O/ab.log "C3 C4" "base P F" 2 || exit 1
bash profiles/ab.sh $O/ab_c5.log "C5" "base P" 1 || exit 1
B="python bench.py --config C3 --steps 1 --warmup 0 --no-cpu-baseline --no-other-configs --pmc off"
for v in base P; do
  if [ $v = base ]; then lib=$PWD/$L/build/librtx_hip.so; else lib=$PWD/$L/build_dbg$v/librtx_hip.so; fi
  RTX_LIB=$lib timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d $O/pmc_${v}_a -o C3 -- $B > $O/pmc_${v}_a.log 2>&1 || { tail -20 $O/pmc_${v}_a.log; exit 1; }
  RTX_LIB=$lib timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_${v}_b -o C3 -- $B > $O/pmc_${v}_b.log 2>&1 || { tail -20 $O/pmc_${v}_b.log; exit 1; }
done
echo done
