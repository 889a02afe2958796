#!/bin/bash
# PMC passes (tools/pmc_sq.txt) of tools/diag_time.py for several library builds:
#   tools/pmc_ab.sh <tag> <lib-name>...   (libs under vad_amd/lib/, e.g. libvad_amd libvad_amd_v2)
# -> gpurun_out/pmcab_<tag>/<lib>/<pass>/ ; summarise with tools/pmc_summary.py
set -u
TAG=$1; shift
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for L in "$@"; do
  i=0
  while read -r P; do
    [ -z "$P" ] && continue
    OUT=$R/gpurun_out/pmcab_$TAG/$L/$i
    mkdir -p $OUT
    VAD_AMD_LIB=$R/vad_amd/lib/$L.so timeout -s KILL 90 rocprofv3 --pmc $P -d $OUT -o run --output-format csv -- python3 $R/tools/diag_time.py > $OUT/log 2>&1 || exit $?
    i=$((i+1))
  done < $R/${PMC_FILE:-tools/pmc_sq.txt}
done
