#!/bin/bash
# mfcc3 kernel: correctness on the MFCC tests, then A/B against the two-wave build
set -u
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-m3}
mkdir -p $OUT
cd $R
timeout -k 10 600 python3 -u -m pytest -x -v -s --timeout 240 --timeout-method thread \
  tests/test_gpu_fullsize.py tests/test_gpu_parity.py -k "mfcc or c2 or c3 or spec or analyser or framing or module" \
  > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
timeout -k 10 300 python3 tools/ab_mfcc.py $R/vad_amd/lib/libvad_amd_v2.so $R/vad_amd/lib/libvad_amd.so 3 > $OUT/ab.json 2>&1 || { tail -20 $OUT/ab.json; exit 2; }
cat $OUT/ab.json
AB_I16=1 timeout -k 10 300 python3 tools/ab_mfcc.py $R/vad_amd/lib/libvad_amd_v2.so $R/vad_amd/lib/libvad_amd.so 2 > $OUT/ab16.json 2>&1 || { tail -20 $OUT/ab16.json; exit 3; }
cat $OUT/ab16.json
