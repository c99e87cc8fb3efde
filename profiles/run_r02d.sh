# Round 2, pass d: device binned-SAH BVH builder -- its tests, then host SAH /
# device LBVH / device SAH build time, SAH cost and render rate on 100k and 1M
# random spheres.
set -e
export TMPDIR=/tmp
O=gpurun_out/r02d
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_device_bvh.py -x -v -m gpu --timeout 200 --timeout-method thread > $O/device_bvh_tests.log 2>&1 || { tail -40 $O/device_bvh_tests.log; exit 1; }
tail -3 $O/device_bvh_tests.log
timeout -k 10 400 python tools/bvh_build_bench.py --n 100000 1000000 > $O/bvh_build.log 2>&1
cat $O/bvh_build.log
