#!/bin/bash
# round 5: FFN A/B (round-4 HEAD library vs this tree) then the round-end style validation
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 420 python tools/ab_ffn.py vad_amd/lib/libvad_amd_base.so vad_amd/lib/libvad_amd.so 3 > gpurun_out/abffn2.json 2>gpurun_out/abffn2.err && bash tools/validate.sh r05b
