#!/bin/bash
# Quick check after a bench.py change: N = 1 bench line (no CPU / secondary
# legs) and the 2-rank gloo rehearsal of the N > 1 path on the box's one GPU.
set -u
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/quick
mkdir -p $OUT
cd $R
timeout -k 10 200 python3 bench.py --no-cpu --no-secondary > $OUT/bench1.json 2> $OUT/bench1.err || { tail -20 $OUT/bench1.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench1.json'));print('N=1', d['value'], d['ms_per_step'])"
timeout -k 10 150 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29519 bench.py --gpus 2 --backend gloo --steps 20 --warmup 5 --no-cpu --no-secondary \
  > $OUT/bench2.json 2> $OUT/bench2.err || { tail -20 $OUT/bench2.err; exit 2; }
python3 -c "import json;d=json.load(open('$OUT/bench2.json'));print('N=2 gloo', d['value'], d['ms_per_step'], d.get('gather'))"
