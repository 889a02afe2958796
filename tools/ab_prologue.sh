#!/bin/bash
# Round-6 prologue A/B (profiles/r06/prologue_ab): label check of the "pro" build, MFCC
# (base vs pro), FFN (base vs pf0) and pipelined steps (base vs pro); libs built by hand.
set -u
R=$GRAFT_REPO_ROOT; cd $R; OUT=gpurun_out/r06n; mkdir -p $OUT
L=vad_amd/lib
VAD_AMD_LIB=$L/libvad_amd_pro.so timeout -k 10 120 python3 tools/fused_vs_two.py > $OUT/fv.jsonl 2> $OUT/fv.err || { tail -20 $OUT/fv.err; exit 1; }
cat $OUT/fv.jsonl
timeout -k 10 600 python3 tools/ab_mfcc.py $L/libvad_amd_base.so $L/libvad_amd_pro.so 4 > $OUT/ab_mfcc.json 2> $OUT/ab_mfcc.err || { tail -20 $OUT/ab_mfcc.err; exit 2; }
cat $OUT/ab_mfcc.json
timeout -k 10 600 python3 tools/ab_ffn.py $L/libvad_amd_base.so $L/libvad_amd_pf0.so 4 > $OUT/ab_ffn.json 2> $OUT/ab_ffn.err || { tail -20 $OUT/ab_ffn.err; exit 3; }
cat $OUT/ab_ffn.json
timeout -k 10 600 python3 tools/ab_pipe.py $L/libvad_amd_base.so $L/libvad_amd_pro.so 3 > $OUT/ab_pipe.json 2> $OUT/ab_pipe.err || { tail -20 $OUT/ab_pipe.err; exit 4; }
cat $OUT/ab_pipe.json
