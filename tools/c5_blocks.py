"""C5 per-hop time of the one-kernel hop, K hops per launch (direct launches):
VAD_AMD_LIB=... python tools/c5_blocks.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vad_amd.ffn import TOPOLOGY_BL13, FFNClassifier, random_layers  # noqa: E402
from vad_amd.stream import StreamBatch  # noqa: E402

dev = torch.device("cuda", 0)
S = 512
clf = FFNClassifier(random_layers(TOPOLOGY_BL13, seed=3))
res = {}
for K in (1, 8, 32):
    sb = StreamBatch(S, clf, hops_per_step=K)
    g = torch.Generator(device=dev).manual_seed(500)
    sb.prime(torch.randn((S, 240), generator=g, device=dev) * 1000)
    blk = torch.randn((K, S, 160), generator=g, device=dev) * 1000
    sb.inputs.copy_(blk)
    reps = max(40, 800 // K)
    for _ in range(reps):
        sb.step_block()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        sb.step_block()
    e.record()
    torch.cuda.synchronize()
    res[K] = s.elapsed_time(e) / (reps * K) * 1e3
print(json.dumps({"lib": os.path.basename(os.environ.get("VAD_AMD_LIB", "")), "us_per_hop": res}))
