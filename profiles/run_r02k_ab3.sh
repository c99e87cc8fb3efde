set -o pipefail
mkdir -p gpurun_out/r02k
export PYTHONPATH=$PWD/real-time-ray-tracing-engine_amd
for n in 20000 100000; do
  echo "== n=$n default" && timeout -k 10 200 python -u tools/arity_ab.py --no-c3 --n $n --rounds 3 &&
  echo "== n=$n LDS nodes 0" && RTX_LDS_NODES=0 timeout -k 10 200 python -u tools/arity_ab.py --no-c3 --n $n --rounds 3 &&
  echo "== n=$n stack4 default (the 16-entry override was a temporary build)" && timeout -k 10 200 python -u tools/arity_ab.py --no-c3 --n $n --rounds 3 || exit 1
done
