# A/B of hop-kernel launch shapes: python tools/c5_bench.py 512 hop per library variant
set -e
for i in 1 2; do
  for L in "" w4 w8; do
    if [ -z "$L" ]; then export VAD_AMD_LIB=vad_amd/lib/libvad_amd.so; else export VAD_AMD_LIB=vad_amd/lib/libvad_amd_$L.so; fi
    echo "lib=$VAD_AMD_LIB"; timeout -k 10 120 python tools/c5_bench.py 512 hop
  done
done
