#!/bin/bash
set -u
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-m3b}
mkdir -p $OUT
cd $R
timeout -k 10 600 python3 -u -m pytest -x -v -s --timeout 240 --timeout-method thread \
  tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_features_parity.py -k "mfcc or c2 or c3 or spec or analyser or framing or module or rows" \
  > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
L=$R/vad_amd/lib
timeout -k 10 400 python3 tools/ab_mfcc.py $L/libvad_amd_v2.so $L/libvad_amd_m3p0.so $L/libvad_amd.so 3 > $OUT/ab.json 2>&1 || { tail -20 $OUT/ab.json; exit 2; }
cat $OUT/ab.json
timeout -k 10 300 bash tools/pmc_ab.sh ${1:-m3b} libvad_amd > $OUT/pmc.log 2>&1 || { tail $OUT/pmc.log; exit 3; }
