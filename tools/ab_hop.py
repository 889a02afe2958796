"""A/B of the streaming hop kernel (C5: 512 streams, 13-64-64-2) across library
builds, fresh processes alternated: python tools/ab_hop.py LIB_A LIB_B [...] [rounds]

Per build and round, us per hop (median of 5 batches): the one-hop kernel
launched directly on device input (K = 1), K = 8 hops per launch, and the
end-to-end one-hop step with host I/O replayed as one hipGraph
(StreamBatch.step_host); beside them the floor: a one-element torch kernel
launched back to back, and the one-hop kernel for 4 streams (one block); the labels of a fixed 40-hop sequence are compared
with the first build's."""
import json
import os
import subprocess
import sys

import numpy as np

CHILD = r'''
import json, os, sys, torch, numpy as np
sys.path.insert(0, os.getcwd())
from vad_amd.ffn import TOPOLOGY_BL13, FFNClassifier, random_layers
from vad_amd.stream import StreamBatch
dev = torch.device("cuda", 0)
S = 512
clf = FFNClassifier(random_layers(TOPOLOGY_BL13, seed=3))
g = torch.Generator(device=dev).manual_seed(500)
prime = torch.randn((S, 240), generator=g, device=dev) * 1000
blocks = [torch.randn((8, S, 160), generator=g, device=dev) * 1000 for _ in range(5)]
def timed(one, K, batches=5, reps=100):
    for k in range(100): one(k)
    torch.cuda.synchronize()
    ts = []
    for _ in range(batches):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for k in range(reps): one(k)
        e.record(); torch.cuda.synchronize()
        ts.append(s.elapsed_time(e) / (reps * K) * 1e3)
    return sorted(ts)[batches // 2]
out = {}
x1 = torch.zeros(1, device=dev)
out["launch_floor_us"] = timed(lambda k: x1.add_(1.0), 1)  # one tiny torch kernel, back to back
s4 = StreamBatch(4, clf); s4.prime(prime[:4])
out["s4_k1_direct_us"] = timed(lambda k: s4.step(blocks[k % 5][k % 8][:4]), 1)
sb = StreamBatch(S, clf); sb.prime(prime)
out["k1_direct_us"] = timed(lambda k: sb.step(blocks[k % 5][k % 8]), 1)
sb8 = StreamBatch(S, clf, hops_per_step=8); sb8.prime(prime)
out["k8_direct_us"] = timed(lambda k: sb8.step_block(blocks[k % 5]), 8, reps=25)
sh = StreamBatch(S, clf); sh.prime(prime); sh.capture(host_io=True)
sh.host_inputs.copy_(blocks[0][:1].cpu())
out["k1_e2e_graph_us"] = timed(lambda k: sh.step_host(), 1)
ref = StreamBatch(S, clf); ref.prime(prime)
labs = [ref.step(blocks[t // 8][t % 8]).cpu().numpy().copy() for t in range(40)]
np.save(os.environ["AB_OUT"] + "_hop.npy", np.stack(labs))
print(json.dumps(out))
'''

args = sys.argv[1:]
rounds = int(args.pop()) if args and args[-1].isdigit() else 3
os.makedirs("gpurun_out", exist_ok=True)
res = {l: [] for l in args}
for r in range(rounds):
    for i, l in enumerate(args):
        env = dict(os.environ, VAD_AMD_LIB=l, AB_OUT=f"gpurun_out/abhop_{i}")
        p = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
        line = [x for x in p.stdout.splitlines() if x.startswith("{")]
        res[l].append(json.loads(line[-1]) if line else {"error": p.stderr[-400:]})
summary = {}
for i, l in enumerate(args):
    d = {}
    for k in ("launch_floor_us", "s4_k1_direct_us", "k1_direct_us", "k8_direct_us", "k1_e2e_graph_us"):
        xs = sorted(x[k] for x in res[l] if k in x)
        d[k] = xs[len(xs) // 2] if xs else None
        d[k + "_all"] = [round(x, 2) for x in xs]
    a = np.load("gpurun_out/abhop_0_hop.npy")
    b = np.load(f"gpurun_out/abhop_{i}_hop.npy")
    d["labels_differ_from_first"] = int((a != b).sum())
    summary[os.path.basename(l)] = d
print(json.dumps(summary))
