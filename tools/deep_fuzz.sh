#!/bin/bash
# Deep fuzz passes (tests/test_gpu_fuzz.py): the derandomized suite, then
# VAD_FUZZ_SCALE x the examples from each seed given.  tools/deep_fuzz.sh <scale> <seed>...
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/deepfuzz
SCALE=$1; shift
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_fuzz.py -q --timeout 240 --timeout-method thread \
  > gpurun_out/deepfuzz/default.log 2>&1 || { tail -60 gpurun_out/deepfuzz/default.log; exit 1; }
tail -1 gpurun_out/deepfuzz/default.log
for S in "$@"; do
  VAD_FUZZ_SCALE=$SCALE VAD_FUZZ_SEED=$S timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fuzz.py -q \
    --timeout 500 --timeout-method thread > gpurun_out/deepfuzz/seed_$S.log 2>&1
  rc=$?
  echo "seed $S rc=$rc: $(tail -1 gpurun_out/deepfuzz/seed_$S.log)"
  case $rc in 0|1) ;; *) tail -40 gpurun_out/deepfuzz/seed_$S.log; exit $rc;; esac
done
