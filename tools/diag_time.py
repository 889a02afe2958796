"""Time mfcc_kernel (1M frames) for the VAD_DIAG ablation set in the env."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import synth_audio  # noqa: E402
from vad_amd.pipeline import VadPipeline  # noqa: E402

pipe = VadPipeline()
F = 1_000_000
audio = synth_audio(160 * (F - 1) + 401, 1, torch.device("cuda"))
out = torch.zeros((F, 13), dtype=torch.float32, device="cuda")
for _ in range(3):
    pipe.mfcc(audio, out=out)
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
n = 20
s.record()
for _ in range(n):
    pipe.mfcc(audio, out=out)
e.record()
torch.cuda.synchronize()
tag = " ".join(f"{k}={v}" for k, v in os.environ.items() if k.startswith("VAD_"))
print(f"[{tag}] mfcc {s.elapsed_time(e) / n * 1e3:.1f} us")
