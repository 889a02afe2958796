"""[Historical: the diagnostic hooks this needs were removed from the shipped kernels in round 4;
build it from a tree at or before commit 4f8ce33.]  Phase timing of mfcc_kernel from in-kernel s_memtime stamps (a -DVAD_DIAG_BUILD=5 library)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
# the stamps come from a diagnostic library build (the shipped one has none):
#   python -m vad_amd.build --variant diag5 -DVAD_DIAG_BUILD=5
os.environ.setdefault("VAD_AMD_LIB", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                  "vad_amd", "lib", "libvad_amd_diag5.so"))
os.environ.setdefault("VAD_DIAG", "5")  # read by this script only
from bench import synth_audio  # noqa: E402
from vad_amd.pipeline import VadPipeline  # noqa: E402

pipe = VadPipeline()
F = 1_000_000
audio = synth_audio(160 * (F - 1) + 401, 1, torch.device("cuda"))
if os.environ.get("VAD_STAMP_INT16"):
    audio = audio.to(torch.int16)
out = torch.zeros((F, 13), dtype=torch.float32, device="cuda")
for _ in range(3):
    pipe.mfcc(audio, out=out)
torch.cuda.synchronize()
st = out.reshape(-1).view(torch.int64)[: 256 * 8 * 8 * 16].cpu().numpy().reshape(256, 8, 8, 16)
waves = range(8) if os.environ["VAD_DIAG"] in ("5", "8") else range(4)
st = st[:, list(waves), 1:7, :11]  # skip the first tile (cold), keep tiles 1..6
d = np.diff(st.astype(np.float64), axis=-1)  # 10 intervals
names = ["stageA_A", "xposeA", "stageA_B", "finish_A", "xposeB", "finish_B", "phase2b", "bar1",
         "phase2a", "bar2"]
tot = np.median(st[..., 10] - st[..., 0])
print(f"VAD_DIAG={os.environ['VAD_DIAG']}: median cycles per tile {tot:.0f}")
for i, n in enumerate(names):
    print(f"{n:9s}", [int(np.median(d[:, w, :, i])) for w in range(len(waves))])
