#!/bin/bash
# A/B of bench.py's pipelined step: --streams 1 vs 2 vs 3, interleaved, plus
# the alternating-stream label test.  Writes gpurun_out/streams_ab/.
set -u
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/streams_ab
mkdir -p $OUT
cd $R
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_fullsize.py -k alternating -x -v --timeout 200 --timeout-method thread > $OUT/test.log 2>&1 || { tail -30 $OUT/test.log; exit 1; }
tail -3 $OUT/test.log
for r in 1 2 3; do
  for s in 1 2 3; do
    timeout -k 10 200 python3 bench.py --no-cpu --no-secondary --streams $s > $OUT/bench_s${s}_r${r}.json 2>> $OUT/bench.err || exit 3
    python3 -c "import json;d=json.load(open('$OUT/bench_s${s}_r${r}.json'));print('streams',$s,'round',$r,'%.4f ms/step'%d['ms_per_step'],'%.3e'%d['value'])"
  done
done
