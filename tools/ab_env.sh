#!/bin/bash
# A/B kernel timing of runtime variants selected by environment assignments:
#   tools/ab_env.sh "VAD_X=0" "VAD_X=1" ...   (two rounds, fp32 and int16 input)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
for round in 1 2; do
  for v in "$@"; do
    for dt in f32 i16; do
      if [ $dt = i16 ]; then export VAD_DIAG_INT16=1; else unset VAD_DIAG_INT16; fi
      env $v timeout -k 10 120 python3 $R/tools/diag_time.py 2>&1 | grep -v amdgpu.ids || exit $?
    done
  done
done
