set -e
AB_I16=1 timeout -k 10 300 python tools/ab_mfcc.py vad_amd/lib/libvad_amd_h.so vad_amd/lib/libvad_amd.so 2 > gpurun_out/r02_ab_raw16.json
AB_I16=1 timeout -k 10 300 python tools/ab_mfcc.py vad_amd/lib/libvad_amd.so vad_amd/lib/libvad_amd_p16.so 2 > gpurun_out/r02_ab_raw16p.json
timeout -k 10 300 python tools/ab_mfcc.py vad_amd/lib/libvad_amd_h.so vad_amd/lib/libvad_amd.so 2 > gpurun_out/r02_ab_raw32.json
