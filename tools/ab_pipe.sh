#!/bin/bash
# Label check (fused vs two-kernel vs oracle) per library variant, then the
# pipelined-step A/B: tools/ab_pipe.sh <tag> <rounds> NAME...  (vad_amd/lib/libvad_amd_NAME.so)
set -u
TAG=$1; N=$2; shift 2
R=$GRAFT_REPO_ROOT; cd $R; OUT=gpurun_out/$TAG; mkdir -p $OUT
for v in "$@"; do
  VAD_AMD_LIB=vad_amd/lib/libvad_amd_$v.so timeout -k 10 120 python3 tools/fused_vs_two.py >> $OUT/fv.jsonl 2>> $OUT/fv.err || { tail -20 $OUT/fv.err; exit 1; }
done
cat $OUT/fv.jsonl
LIBS=""; for v in "$@"; do LIBS="$LIBS vad_amd/lib/libvad_amd_$v.so"; done
timeout -k 10 600 python3 tools/ab_ffn.py $LIBS 2 > $OUT/ab_ffn.json 2> $OUT/ab_ffn.err || { tail -20 $OUT/ab_ffn.err; exit 2; }
cat $OUT/ab_ffn.json
timeout -k 10 900 python3 tools/ab_pipe.py $LIBS $N > $OUT/ab_pipe.json 2> $OUT/ab_pipe.err || { tail -20 $OUT/ab_pipe.err; exit 3; }
cat $OUT/ab_pipe.json
