#!/bin/bash
# Round 4 first GPU call: the matrix-core phase-1 prototype, then the round-end style validation.
set -u
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r04a
cd $R
timeout -k 10 60 bin_tmp/mx_proto > gpurun_out/r04a/mx_proto.txt 2>&1; rc=$?
cat gpurun_out/r04a/mx_proto.txt
timeout -k 10 60 bin_tmp/mx_proto 1000000 f >> gpurun_out/r04a/mx_proto.txt 2>&1; rc2=$?
tail -2 gpurun_out/r04a/mx_proto.txt
case $rc in 0|1) ;; *) exit 10;; esac
case $rc2 in 0|1) ;; *) exit 11;; esac
bash tools/validate.sh r04a
