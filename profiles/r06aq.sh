#!/bin/bash
# r06aq: bench.py starting its own 4 and 8 ranks on this one GPU (gloo,
# --share-device, --check against a one-device frame): the launcher and the
# tile-shard exchange at the driver's rank counts
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06aq
mkdir -p $O
for n in 4 8; do
  timeout -k 10 300 python bench.py --gpus $n --backend gloo --share-device --config C2 --steps 3 --warmup 1 --check > $O/launcher_${n}rank_C2.json 2> $O/launcher_${n}rank_C2.err || { tail -20 $O/launcher_${n}rank_C2.err; exit 1; }
  tail -1 $O/launcher_${n}rank_C2.json | cut -c1-260
done
echo done
