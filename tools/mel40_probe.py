"""MFCC kernel time per launch at 26 vs 40 mel filters, 1M and 100k frames
(HIP events around back-to-back launches): python tools/mel40_probe.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import synth_audio  # noqa: E402
from vad_amd.config import MfccConfig  # noqa: E402
from vad_amd.pipeline import VadPipeline  # noqa: E402

dev = torch.device("cuda", 0)


def t(fn, reps=60, warm=100):
    for _ in range(warm):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


res = {}
for F in (1_000_000, 100_000):
    clips = [synth_audio(160 * (F - 1) + 401, 10 + i, dev) for i in range(2 if F > 500_000 else 6)]
    m = torch.empty((F, 13), device=dev)
    for nf in (26, 40):
        pipe = VadPipeline(cfg=MfccConfig(n_filters=nf))
        k = [0]

        def f():
            pipe.mfcc(clips[k[0] % len(clips)], out=m)
            k[0] += 1
        res[f"{F}_{nf}mel_us"] = t(f)
    del clips
print(json.dumps(res))
