set -o pipefail
mkdir -p gpurun_out/r05e
bash profiles/ab.sh gpurun_out/r05e/kb_ab.log "C4 C3 C2" "base C" 2 || exit 1
timeout -k 10 200 python bench.py --config C4 --steps 2 --warmup 1 --no-cpu-baseline --pmc off --no-other-configs > gpurun_out/r05e/bench_C4.json 2> gpurun_out/r05e/bench_C4.err || exit 1
