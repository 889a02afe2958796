#!/bin/bash
# Round-end style validation on the GPU box: GPU test suite, smoke, default bench.
#   tools/validate.sh <tag>
# Writes gpurun_out/val_<tag>/{tests.log,smoke.log,bench.json}; each step has its own timeout.
set -u
TAG=$1
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/val_$TAG
mkdir -p $OUT
cd $R
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -30 $OUT/smoke.log; exit 2; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 3; }
cat $OUT/bench.json
