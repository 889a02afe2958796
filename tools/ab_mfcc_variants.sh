#!/bin/bash
# A/B of library variants (vad_amd/lib/libvad_amd_<name>.so): tools/ab_mfcc_variants.sh <tag> <rounds> <name>...
set -u
TAG=$1; N=$2; shift 2
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/$TAG
LIBS=""
for v in "$@"; do LIBS="$LIBS $R/vad_amd/lib/libvad_amd_$v.so"; done
timeout -k 10 900 python3 tools/ab_mfcc.py $LIBS $N > gpurun_out/$TAG/ab.json 2>&1 || { tail -20 gpurun_out/$TAG/ab.json; exit 2; }
cat gpurun_out/$TAG/ab.json
