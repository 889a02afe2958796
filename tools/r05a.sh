set -o pipefail
mkdir -p gpurun_out
timeout -k 10 420 python tools/ab_ffn.py vad_amd/lib/libvad_amd_base.so vad_amd/lib/libvad_amd.so 3 > gpurun_out/abffn1.json 2>gpurun_out/abffn1.err &&
timeout -k 10 300 python tools/ab_hop.py vad_amd/lib/libvad_amd_base.so vad_amd/lib/libvad_amd.so 2 > gpurun_out/abhop1.json 2>gpurun_out/abhop1.err &&
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_fused.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py -k "fused or c3_full or split_f16 or alternating or stream or hop or c5" > gpurun_out/t_r05a.log 2>&1
