# Round 2, pass f: PC sampling (rocprofv3 beta, host-trap) of the C4 render kernel.
set -e
export TMPDIR=/tmp
O=gpurun_out/r02f
mkdir -p $O
timeout -s KILL 60 rocprofv3 -L > $O/list_avail.txt 2>&1 || true
grep -i -A12 "pc_sampl\|PC sampling" $O/list_avail.txt | head -40 || true
timeout -s KILL 150 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time --pc-sampling-interval 1000 --output-format csv -d $O/pcs_C4 -o pcs -- python bench.py --config C4 --steps 1 --warmup 0 --no-cpu-baseline --pmc off --no-other-configs > $O/pcs_C4.log 2>&1
ls -la $O/pcs_C4/*/* 2>/dev/null | head; find $O/pcs_C4 -name "*.csv" | head
