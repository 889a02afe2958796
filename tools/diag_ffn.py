"""Time the FFN window kernel (features + MLP) on 1M MFCC rows: min / median
of 5 batches of 20 launches.  VAD_FFN_TOPO=ref39 for the Keras topology."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import synth_audio  # noqa: E402
from vad_amd.ffn import TOPOLOGY_BL13, TOPOLOGY_REF39, FFNClassifier, random_layers  # noqa: E402
from vad_amd.pipeline import VadPipeline  # noqa: E402

topo = {"ref39": TOPOLOGY_REF39, "bl13c3": (13, 64, 64, 3)}.get(os.environ.get("VAD_FFN_TOPO"),
                                                                TOPOLOGY_BL13)
pipe = VadPipeline(FFNClassifier(random_layers(topo, seed=3)))
F = 1_000_000
audio = synth_audio(160 * (F - 1) + 401, 1, torch.device("cuda"))
mfcc = pipe.mfcc(audio)
labels = torch.empty((F - 5,), dtype=torch.uint8, device="cuda")
plan = pipe.ffn.plan
for _ in range(150):  # past the clock ramp of a cold GPU
    plan.window_labels(mfcc, out=labels)
ts = []
for _ in range(5):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(20):
        plan.window_labels(mfcc, out=labels)
    e.record()
    torch.cuda.synchronize()
    ts.append(s.elapsed_time(e) / 20 * 1e3)
ts.sort()
tag = " ".join(f"{k}={v}" for k, v in os.environ.items() if k.startswith("VAD_") and k != "VAD_AMD_LIB")
print(f"[{tag}] ffn min {ts[0]:.1f} us  median {ts[2]:.1f} us  labels {torch.bincount(labels).tolist()}")
