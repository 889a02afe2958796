"""Time mfcc_kernel (1M frames) of the library VAD_AMD_LIB names (A/B of
variant builds: python -m vad_amd.build --variant NAME -D...)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import synth_audio  # noqa: E402
from vad_amd.pipeline import VadPipeline  # noqa: E402

pipe = VadPipeline()
F = 1_000_000
audio = synth_audio(160 * (F - 1) + 401, 1, torch.device("cuda"))
if os.environ.get("VAD_DIAG_INT16"):
    audio = audio.to(torch.int16)
out = torch.zeros((F, 13), dtype=torch.float32, device="cuda")
for _ in range(150):  # past the clock ramp of a cold GPU
    pipe.mfcc(audio, out=out)
ts = []
for _ in range(5):  # 5 batches of 20 launches: min and median of the batch means
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 20
    s.record()
    for _ in range(n):
        pipe.mfcc(audio, out=out)
    e.record()
    torch.cuda.synchronize()
    ts.append(s.elapsed_time(e) / n * 1e3)
ts.sort()
tag = " ".join(f"{k}={v}" for k, v in os.environ.items() if k.startswith("VAD_") and k != "VAD_AMD_LIB")
chk = out.double().abs().sum().item()  # variants must agree exactly
print(f"[{tag}] mfcc min {ts[0]:.1f} us  median {ts[2]:.1f} us  checksum {chk:.17g}")
