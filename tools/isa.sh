#!/bin/bash
# Device assembly of one translation unit with the library's flags for that
# unit (vad_amd/build.py: the common flags plus UNIT_FLAGS[unit]):
#   tools/isa.sh mfcc_kernel.hip /tmp/out.s [extra hipcc flags]
set -e
U=$1; O=$2; shift 2
cd "$(dirname "$0")/.."
UF=$(python3 -c "import sys; from vad_amd.build import UNIT_FLAGS; print(' '.join(UNIT_FLAGS.get(sys.argv[1], [])))" "$U")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Iinclude $UF \
  --cuda-device-only -S "$@" vad_amd/csrc/$U -o "$O"
