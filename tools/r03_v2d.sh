#!/bin/bash
set -u
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-v2d}
mkdir -p $OUT
cd $R
timeout -k 10 600 python3 -u -m pytest -x -v -s --timeout 240 --timeout-method thread \
  tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_fused.py tests/test_gpu_stages.py tests/test_gpu_features_parity.py \
  > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
timeout -k 10 600 bash tools/r03_ab.sh ${1:-v2d} 3 v2v m3c main > $OUT/ab.log 2>&1 || { tail -5 $OUT/ab.log; exit 2; }
