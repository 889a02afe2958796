"""Per-1M-frame time of the MFCC stage with the optional pre-emphasis / Hamming
stages on and off (north_star names them; the reference has neither)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import synth_audio  # noqa: E402
from vad_amd.config import MfccConfig  # noqa: E402
from vad_amd.pipeline import VadPipeline  # noqa: E402

F = 1_000_000
dev = torch.device("cuda")
a = synth_audio(160 * (F - 1) + 401, 1, dev)
m = torch.empty((F, 13), device=dev)
res = {}
for name, cfg in (("off", MfccConfig()), ("hamming", MfccConfig(window="hamming")),
                  ("preemph", MfccConfig(preemph=0.97)), ("both", MfccConfig(preemph=0.97, window="hamming"))):
    pipe = VadPipeline(cfg=cfg)
    for _ in range(30):
        pipe.mfcc(a, out=m)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(50):
        pipe.mfcc(a, out=m)
    e.record()
    torch.cuda.synchronize()
    res[name] = s.elapsed_time(e) / 50 * 1e3
print(json.dumps({"us_per_1M_frames": res}))
