set -o pipefail
mkdir -p gpurun_out/r05b
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 60 rocprofv3 -L > gpurun_out/r05b/list_avail.txt 2>&1
grep -i -B2 -A12 "pc.sampl\|PC_SAMPL" gpurun_out/r05b/list_avail.txt | head -60
timeout -s KILL 150 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic --pc-sampling-unit cycles --pc-sampling-interval 65536 -d gpurun_out/r05b/pcs -o pcs --output-format csv -- python bench.py --config C4 --width 960 --spp 64 --steps 1 --warmup 1 --no-cpu-baseline --pmc off --no-other-configs > gpurun_out/r05b/pcs.log 2>&1
echo rc=$?
tail -5 gpurun_out/r05b/pcs.log
find gpurun_out/r05b/pcs -type f | head; 
