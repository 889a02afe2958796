"""Fused vs two-kernel clip labels on the C host test's clip (30k frames,
seed 71, 13-64-64-2 seed 5) for one library (VAD_AMD_LIB), against the
oracle: python tools/fused_vs_two.py  -> one JSON line."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import vad_oracle as O  # noqa: E402
from vad_amd.ffn import TOPOLOGY_BL13, FFNClassifier, random_layers  # noqa: E402
from vad_amd.pipeline import VadPipeline  # noqa: E402

F = int(os.environ.get("FV_FRAMES", "30000"))
clip = O.synth_clip(O.samples_for_frames(F), seed=int(os.environ.get("FV_SEED", "71")))
layers = random_layers(TOPOLOGY_BL13, seed=5)
pipe = VadPipeline(FFNClassifier(layers))
a = torch.from_numpy(clip).cuda()
two = pipe.labels(a).cpu().numpy()
fused = pipe.labels(a, fused=True).cpu().numpy()
m = pipe.mfcc(a).cpu().numpy()
x = O.analyser_features_fast(m.astype(np.float64))[:, :13]
ref = O.ffn_labels(x, layers)
marg = O.ffn_margin(x, layers)
sure = marg > 1e-4
bad = np.flatnonzero(two != fused)
print(json.dumps({"lib": os.environ.get("VAD_AMD_LIB", "default"), "windows": int(len(two)),
                  "fused_ne_two": int(len(bad)), "first": bad[:10].tolist(),
                  "two_ne_oracle_sure": int((two[sure] != ref[sure]).sum()),
                  "fused_ne_oracle_sure": int((fused[sure] != ref[sure]).sum()),
                  "two_head": two[:12].tolist(), "fused_head": fused[:12].tolist(), "ref_head": ref[:12].tolist()}))
