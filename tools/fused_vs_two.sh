set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/dbg
for L in rowclamp bufrows pf2; do
  VAD_AMD_LIB=vad_amd/lib/libvad_amd_$L.so timeout -k 10 120 python3 tools/fused_vs_two.py >> gpurun_out/dbg/fv.jsonl 2>> gpurun_out/dbg/fv.err || exit 1
done
cat gpurun_out/dbg/fv.jsonl
