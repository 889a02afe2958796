"""Phase timing of mfcc_kernel from in-kernel s_memtime stamps (VAD_DIAG=5)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["VAD_DIAG"] = "5"
from bench import synth_audio  # noqa: E402
from vad_amd.pipeline import VadPipeline  # noqa: E402

pipe = VadPipeline()
F = 1_000_000
audio = synth_audio(160 * (F - 1) + 401, 1, torch.device("cuda"))
out = torch.zeros((F, 13), dtype=torch.float32, device="cuda")
for _ in range(3):
    pipe.mfcc(audio, out=out)
torch.cuda.synchronize()
st = out.reshape(-1).view(torch.int64)[: 256 * 8 * 8 * 8].cpu().numpy().reshape(256, 8, 8, 8)
st = st[:, :, 1:7, :]  # skip first tile (cold), keep iterations 1..6
d = np.diff(st[..., :7].astype(np.float64), axis=-1)  # 6 intervals
names = ["pass0", "pass1", "phase2b", "bar1", "phase2a", "bar2"]
tot = d.sum(axis=-1)
print("cycles per tile (median over blocks/waves/iters):", np.median(tot))
for i, n in enumerate(names):
    print(f"{n:8s} median {np.median(d[..., i]):8.0f}  mean {d[..., i].mean():8.0f}  "
          f"share {d[..., i].mean() / tot.mean():.3f}")
for i, n in enumerate(names):
    print(f"per-wave {n} medians:", [int(np.median(d[:, w, :, i])) for w in range(8)])
