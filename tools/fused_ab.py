"""A/B: fused clip kernel (vad_mfcc_ffn) vs the two-kernel form, 1M frames.

    python tools/fused_ab.py [frames] [reps]

Prints per-launch ms (HIP events around back-to-back launches, batches of 10)
for bl13 / ref39, fp32 / int16 input, and whether the labels agree.
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import synth_audio  # noqa: E402
from vad_amd.ffn import TOPOLOGY_BL13, TOPOLOGY_REF39, FFNClassifier, random_layers  # noqa: E402
from vad_amd.pipeline import VadPipeline  # noqa: E402

F = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
REPS = int(sys.argv[2]) if len(sys.argv) > 2 else 50
dev = torch.device("cuda", 0)
audio = synth_audio(160 * (F - 1) + 401, 100, dev)
audio16 = audio.to(torch.int16)
st = torch.cuda.current_stream()


def timeit(fn, reps=REPS, batch=10):
    for _ in range(20):
        fn()
    nb = max(1, reps // batch)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(nb + 1)]
    ev[0].record(st)
    for i in range(nb):
        for _ in range(batch):
            fn()
        ev[i + 1].record(st)
    torch.cuda.synchronize()
    per = sorted(ev[i].elapsed_time(ev[i + 1]) / batch for i in range(nb))
    return {"mean": ev[0].elapsed_time(ev[nb]) / (nb * batch), "p50": per[nb // 2]}


res = {}
for name, topo in (("bl13", TOPOLOGY_BL13), ("ref39", TOPOLOGY_REF39)):
    pipe = VadPipeline(FFNClassifier(random_layers(topo, seed=3)))
    for tag, a in (("f32", audio), ("i16", audio16)):
        out = torch.empty(F - 5, dtype=torch.uint8, device=dev)
        out2 = torch.empty_like(out)
        fused = timeit(lambda: pipe.labels(a, out=out, fused=True))
        unfused = timeit(lambda: pipe.labels(a, out=out2))
        same = bool(torch.equal(out, out2))
        res[f"{name}_{tag}"] = {"fused_ms": fused, "two_kernel_ms": unfused, "labels_equal": same}
mf = torch.empty((F, 13), dtype=torch.float32, device=dev)
pipe = VadPipeline()
res["mfcc_only_f32_ms"] = timeit(lambda: pipe.mfcc(audio, out=mf))
res["mfcc_only_i16_ms"] = timeit(lambda: pipe.mfcc(audio16, out=mf))
print(json.dumps(res))
