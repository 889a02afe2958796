#!/bin/bash
# A/B of two MFCC libraries (fresh processes, alternating): C3 1M frames, C2 100k at 26 / 40 mel.
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04e
timeout -k 10 500 python3 tools/ab_mfcc.py "$@" > gpurun_out/r04e/ab.json 2>&1 || { tail -20 gpurun_out/r04e/ab.json; exit 1; }
cat gpurun_out/r04e/ab.json
