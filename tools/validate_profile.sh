#!/bin/bash
# Full validation: GPU tests,
# smoke, default bench, the bench's own 2-rank launcher (gloo, one GPU), then
# the kernel trace + PMC passes (tools/profile.sh).  Stops at the first failure.
set -u
TAG=$1
R=$GRAFT_REPO_ROOT
cd $R
bash tools/validate.sh $TAG || exit $?
OUT=$R/gpurun_out/val_$TAG
timeout -k 10 300 python3 bench.py --gpus 2 --backend gloo --steps 20 --warmup 5 --no-cpu --no-secondary \
  > $OUT/bench_2rank_gloo.json 2> $OUT/bench_2rank_gloo.err || { tail -20 $OUT/bench_2rank_gloo.err; exit 9; }
cat $OUT/bench_2rank_gloo.json
bash tools/profile.sh $TAG --steps 5 --warmup 2 --no-cpu --no-secondary || exit 10
echo all done
