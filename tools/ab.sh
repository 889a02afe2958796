#!/bin/bash
# A/B kernel timing of library variants: tools/ab.sh <lib-name>... (under vad_amd/lib/)
# Runs tools/diag_time.py (1M frames, fp32 and int16 input) alternating the libraries.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
for round in 1 2; do
  for v in "$@"; do
    for dt in f32 i16; do
      if [ $dt = i16 ]; then export VAD_DIAG_INT16=1; else unset VAD_DIAG_INT16; fi
      echo -n "$v $dt: "
      VAD_AMD_LIB=$R/vad_amd/lib/$v.so timeout -k 10 120 python3 $R/tools/diag_time.py || exit $?
    done
  done
done
