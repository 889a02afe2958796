#!/bin/bash
# PMC passes over tools/diag_time.py (one rocprofv3 --pmc run per line of the
# passes file): tools/pmc_passes.sh <tag> <passes-file>  -> gpurun_out/pmc_<tag>_<i>/
set -u
TAG=$1; PF=$2
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
i=0
while read -r P; do
  [ -z "$P" ] && continue
  OUT=$R/gpurun_out/pmc_${TAG}_$i
  mkdir -p $OUT
  timeout -k 10 100 rocprofv3 --pmc $P -d $OUT -o run --output-format csv -- python3 $R/${DIAG_SCRIPT:-tools/diag_time.py} > $OUT/log 2>&1 || exit $?
  i=$((i+1))
done < $R/$PF
