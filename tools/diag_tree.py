"""Time the decision-tree window kernel (features + walk) on 1M MFCC rows with
the fixture tree (tests/golden/tree.npz, 977 nodes): min / median of 5
batches of 20 launches, and a checksum of the labels."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from bench import synth_audio  # noqa: E402
from vad_amd.pipeline import VadPipeline  # noqa: E402
from vad_amd.tree import TreeClassifier  # noqa: E402

with np.load(os.path.join(REPO, "tests", "golden", "tree.npz"), allow_pickle=False) as g:
    tree = TreeClassifier(g["feature"], g["threshold"], g["left"], g["right"], g["leaf"],
                          g["nan_left"], g["classes"], int(g["n_features"]))
F = 1_000_000
mfcc = VadPipeline().mfcc(synth_audio(160 * (F - 1) + 401, 1, torch.device("cuda")))
labels = torch.empty((F - 5,), dtype=torch.uint8, device="cuda")
for _ in range(100):
    tree.window_labels(mfcc, out=labels)
ts = []
for _ in range(5):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(20):
        tree.window_labels(mfcc, out=labels)
    e.record()
    torch.cuda.synchronize()
    ts.append(s.elapsed_time(e) / 20 * 1e3)
ts.sort()
print(f"tree min {ts[0]:.1f} us  median {ts[2]:.1f} us  labels {torch.bincount(labels).tolist()}")
