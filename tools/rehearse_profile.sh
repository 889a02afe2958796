#!/bin/bash
# 2-rank gloo rehearsal of bench.py's N > 1 path (both ranks on the box's one
# GPU), then the kernel trace + PMC passes of the default bench.
set -u
TAG=${1:-r03g}
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/val_$TAG
mkdir -p $OUT
timeout -k 10 150 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus 2 --backend gloo --steps 20 --warmup 5 --no-cpu --no-secondary \
  > $OUT/bench_2rank_gloo.json 2> $OUT/bench_2rank_gloo.err || { tail -20 $OUT/bench_2rank_gloo.err; exit 9; }
cat $OUT/bench_2rank_gloo.json
bash tools/profile.sh $TAG --steps 5 --warmup 2 --no-cpu --no-secondary || exit 10
echo all done
