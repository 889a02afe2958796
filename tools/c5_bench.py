"""C5 (BASELINE configs[4]): S concurrent streams, one 10 ms hop per step.
Per-hop time of the streaming forms, HIP events around 400 steps:
  three+graph  push + MFCC + features/FFN kernels captured in one hipGraph
               (the copy of the new samples into the graph's input included)
  hop+graph    the single vad_stream_hop kernel in a hipGraph (copy included)
  hop          the single kernel launched directly on the caller's samples
    python tools/c5_bench.py [S]      (rocprofv3 --kernel-trace --stats -- python3 tools/c5_bench.py)
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vad_amd import ffn as ffn_mod  # noqa: E402
from vad_amd.stream import StreamBatch  # noqa: E402


def per_hop_us(S, kernel, graph, steps=400):
    dev = torch.device("cuda")
    sb = StreamBatch(S, ffn_mod.FFNClassifier(ffn_mod.random_layers(ffn_mod.TOPOLOGY_BL13, seed=3)),
                     kernel=kernel)
    g = torch.Generator(device=dev).manual_seed(500)
    sb.prime(torch.randn((S, 240), generator=g, device=dev) * 1000)
    hops = [torch.randn((S, 160), generator=g, device=dev) * 1000 for _ in range(8)]
    if graph:
        sb.capture()
    for k in range(steps):
        sb.step(hops[k % 8])
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for k in range(steps):
        sb.step(hops[k % 8])
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / steps * 1e3


if __name__ == "__main__":
    S = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    only = sys.argv[2] if len(sys.argv) > 2 else None
    res = {"streams": S}
    for name, kernel, graph in (("three+graph", "three", True), ("hop+graph", "hop", True), ("hop", "hop", False)):
        if only and name != only:
            continue
        us = per_hop_us(S, kernel, graph)
        res[name] = {"us_per_hop": us, "stream_hops_per_s": S / (us * 1e-6),
                     "x_real_time": 10_000.0 / us}
    print(json.dumps(res))
