# A/B of FFN window-kernel library variants: tools/ab_ffn.sh VARIANT... ("" = the shipped library)
set -e
for i in 1 2; do
  for L in "$@"; do
    if [ "$L" = "base" ]; then export VAD_AMD_LIB=vad_amd/lib/libvad_amd.so; else export VAD_AMD_LIB=vad_amd/lib/libvad_amd_$L.so; fi
    echo "lib=$VAD_AMD_LIB"; timeout -k 10 120 python tools/diag_ffn.py
  done
done
