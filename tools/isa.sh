#!/bin/bash
# Device assembly of one translation unit with the library's flags:
#   tools/isa.sh mfcc_kernel.hip /tmp/out.s [extra hipcc flags]
set -e
U=$1; O=$2; shift 2
cd "$(dirname "$0")/.."
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Iinclude \
  -mllvm -amdgpu-sched-strategy=max-ilp --cuda-device-only -S "$@" vad_amd/csrc/$U -o "$O"
