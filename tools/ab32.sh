#!/bin/bash
# A/B kernel timing of library variants, fp32 input only: tools/ab32.sh <lib-name>...
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
for round in 1 2; do
  for v in "$@"; do
    echo -n "$v: "
    VAD_AMD_LIB=$R/vad_amd/lib/$v.so timeout -k 10 120 python3 $R/tools/diag_time.py 2>&1 | grep -v amdgpu.ids || exit $?
  done
done
