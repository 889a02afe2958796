#!/bin/bash
# PMC passes (tools/pmc_ffn.txt, one line per pass) over the bench for each
# library variant: tools/pmc_ffn_ab.sh <tag> NAME...  (vad_amd/lib/libvad_amd_NAME.so)
set -u
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/$TAG; mkdir -p $OUT
cd $R
for v in "$@"; do
  i=0
  while read -r CTRS; do
    i=$((i + 1))
    VAD_AMD_LIB=vad_amd/lib/libvad_amd_$v.so timeout -s KILL 120 rocprofv3 --pmc $CTRS -d $OUT/$v/p$i -o run \
      --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu > $OUT/$v.p$i.log 2>&1 || { tail -20 $OUT/$v.p$i.log; exit 1; }
  done < tools/pmc_ffn.txt
done
python3 tools/pmc_ffn_report.py $OUT "$@" > $OUT/report.json && cat $OUT/report.json
for v in "$@"; do rm -rf $OUT/$v; done  # the raw counter CSVs exceed what gpurun copies back
