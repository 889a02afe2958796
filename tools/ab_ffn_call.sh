#!/bin/bash
# GPU suite, then an FFN window-kernel A/B of library variants:
#   tools/ab_ffn_call.sh <tag> <rounds> NAME...   (vad_amd/lib/libvad_amd_NAME.so)
set -u
TAG=$1; N=$2; shift 2
R=$GRAFT_REPO_ROOT; cd $R; OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
LIBS=""; for v in "$@"; do LIBS="$LIBS vad_amd/lib/libvad_amd_$v.so"; done
timeout -k 10 900 python3 tools/ab_ffn.py $LIBS $N > $OUT/ab_ffn.json 2> $OUT/ab_ffn.err || { tail -20 $OUT/ab_ffn.err; exit 2; }
cat $OUT/ab_ffn.json
