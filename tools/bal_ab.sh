#!/bin/bash
# XCD-balance A/B on one box: per-XCD speeds the balance sees (debug line),
# then tools/ab_mfcc.py with the equal-split variant (libvad_amd_nobal.so,
# -DVAD_BALANCE_DEFAULT=0) against the shipped library.  tools/bal_ab.sh <tag>
set -u
TAG=$1
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/$TAG
VAD_MFCC_BALANCE_DEBUG=100 timeout -k 10 200 python3 tools/mel40_probe.py > gpurun_out/$TAG/probe.json 2> gpurun_out/$TAG/speeds.txt || exit 1
grep balance gpurun_out/$TAG/speeds.txt | head -3
cp vad_amd/lib/libvad_amd.so vad_amd/lib/libvad_amd_bal.so
bash tools/ab_mfcc_variants.sh $TAG 3 nobal bal
