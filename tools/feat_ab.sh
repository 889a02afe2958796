#!/bin/bash
# FFN feature-path A/B: the rsq scale check, the GPU suite on the variant
# library, then diag_ffn (FFN kernel alone, both topologies) and the default
# bench (--no-cpu --no-secondary), base vs variant interleaved.
#   tools/feat_ab.sh VARIANT     (vad_amd/lib/libvad_amd_VARIANT.so vs libvad_amd_base.so)
set -u
V=$1
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/feat_ab_$V
mkdir -p $OUT
cd $R
timeout -k 10 60 tools/checks/rsq_scale_check > $OUT/rsq.txt 2>&1; echo "rsq check rc=$?"; cat $OUT/rsq.txt
VAD_AMD_LIB=vad_amd/lib/libvad_amd_$V.so timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for r in 1 2 3; do
  for L in base $V; do
    for T in bl13 ref39; do
      VAD_FFN_TOPO=$T VAD_AMD_LIB=vad_amd/lib/libvad_amd_$L.so timeout -k 10 120 python3 tools/diag_ffn.py 2>>$OUT/err.log | sed "s/^/$L $T: /" | tee -a $OUT/diag.txt || exit 3
    done
  done
done
for r in 1 2 3; do
  for L in base $V; do
    VAD_AMD_LIB=vad_amd/lib/libvad_amd_$L.so timeout -k 10 200 python3 bench.py --no-cpu --no-secondary > $OUT/bench_${L}_r$r.json 2>>$OUT/err.log || exit 4
    python3 -c "import json;d=json.load(open('$OUT/bench_${L}_r$r.json'));k=d['kernels_ms'];print('$L r$r', '%.4f ms/step'%d['ms_per_step'], 'mfcc %.1f ffn %.1f fused %.1f us'%(k['mfcc_kernel']*1e3,k['ffn_kernel']*1e3,k['mfcc_ffn_fused_kernel']*1e3))" | tee -a $OUT/bench.txt
  done
done
