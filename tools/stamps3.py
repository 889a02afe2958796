"""[Historical: the diagnostic hooks this needs were removed from the shipped kernels in round 4;
build it from a tree at or before commit 4f8ce33.]  Phase timing of mfcc3_kernel from in-kernel s_memtime stamps (a -DVAD_MFCC3=1 -DVAD_M3_DIAG=5 build):
VAD_AMD_LIB=... python tools/stamps3.py"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import synth_audio  # noqa: E402
from vad_amd.pipeline import VadPipeline  # noqa: E402

pipe = VadPipeline()
F = 1_000_000
audio = synth_audio(160 * (F - 1) + 401, 1, torch.device("cuda"))
out = torch.zeros((F, 13), dtype=torch.float32, device="cuda")
for _ in range(20):
    pipe.mfcc(audio, out=out)
torch.cuda.synchronize()
W = int(os.environ.get("STAMP_WAVES", "12"))
st = out.reshape(-1).view(torch.int64)[: 256 * W * 8 * 16].cpu().numpy().reshape(256, W, 8, 16)
st = st[:, :, 1:7, :9].astype(np.float64)  # tiles 1..6
d = np.diff(st, axis=-1)
names = ["stageA0", "store+fin0", "stageA1", "store+fin1", "dct", "bar1", "phase2a", "bar2"]
print(f"median cycles per tile {np.median(st[..., 8] - st[..., 0]):.0f}")
print("phase     " + " ".join(f"w{w:<5d}" for w in range(W)))
for i, n in enumerate(names):
    print(f"{n:10s}" + " ".join(f"{int(np.median(d[:, w, :, i])):6d}" for w in range(W)))
