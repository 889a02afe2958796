#!/bin/bash
# round 5: the 64-window FFN kernel variant -- label tests on it, then the FFN A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
VAD_AMD_LIB=$PWD/vad_amd/lib/libvad_amd_w64.so timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_fused.py tests/test_gpu_features_parity.py \
  -k "c3_full or window_labels or ffn or fused or features or analyser or alternating" > gpurun_out/t_w64.log 2>&1 &&
timeout -k 10 420 python tools/ab_ffn.py vad_amd/lib/libvad_amd_r05b.so vad_amd/lib/libvad_amd_w64.so 3 > gpurun_out/abffn3.json 2>gpurun_out/abffn3.err
