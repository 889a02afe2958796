#!/bin/bash
# round 5: hop kernel with unrolled mel / DCT / FFN loops and a cross-lane
# output layer (variant hop2) -- stream tests on it, then the hop A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
VAD_AMD_LIB=$PWD/vad_amd/lib/libvad_amd_hop2.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_fullsize.py tests/test_gpu_parity.py -k "stream or hop or c5" > gpurun_out/t_hop2.log 2>&1 &&
timeout -k 10 400 python tools/ab_hop.py vad_amd/lib/libvad_amd_r05b.so vad_amd/lib/libvad_amd_hop2.so 3 > gpurun_out/abhop3.json 2>gpurun_out/abhop3.err
