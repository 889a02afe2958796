"""C5 (512 streams, one hop per hipGraph replay) for a rocprofv3 kernel trace:
    rocprofv3 --kernel-trace --stats -d gpurun_out/c5 -- python3 tools/c5_trace.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vad_amd import ffn as ffn_mod  # noqa: E402
from vad_amd.stream import StreamBatch  # noqa: E402

S = int(os.environ.get("C5_STREAMS", "512"))
dev = torch.device("cuda")
sb = StreamBatch(S, ffn_mod.FFNClassifier(ffn_mod.random_layers(ffn_mod.TOPOLOGY_BL13, seed=3)))
g = torch.Generator(device=dev).manual_seed(500)
sb.prime(torch.randn((S, 240), generator=g, device=dev) * 1000)
hops = [torch.randn((S, 160), generator=g, device=dev) * 1000 for _ in range(8)]
sb.capture()
for k in range(400):
    sb.step(hops[k % 8])
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for k in range(400):
    sb.step(hops[k % 8])
e.record()
torch.cuda.synchronize()
print(f"C5 S={S}: {s.elapsed_time(e) / 400 * 1e3:.1f} us per hop")
