#!/bin/bash
# A/B of FFN library variants (tools/ab_ffn.sh): base vs the given variant names.
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04g
timeout -k 10 600 bash tools/ab_ffn.sh base "$@" > gpurun_out/r04g/ab_ffn.txt 2>&1 || { tail -20 gpurun_out/r04g/ab_ffn.txt; exit 1; }
cat gpurun_out/r04g/ab_ffn.txt
