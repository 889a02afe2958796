#!/bin/bash
# A/B FFN window-kernel timing of library variants: tools/ab_ffn.sh <lib-name>...
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
for v in "$@"; do
  for topo in ${TOPOS:-bl13 ref39}; do
    echo -n "$v $topo: "
    VAD_FFN_TOPO=$topo VAD_AMD_LIB=$R/vad_amd/lib/$v.so timeout -k 10 120 python3 $R/tools/diag_ffn.py || exit $?
  done
done
