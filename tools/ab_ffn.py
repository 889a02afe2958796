"""A/B of the FFN window kernel across library builds, fresh processes
alternated: python tools/ab_ffn.py LIB_A LIB_B [...] [rounds]

Per build and round: the 13-64-64-2 (and 39-64-32-16-3) window kernel on the
MFCC rows of the C3 clip (1M frames), median of 7 batches of 20 launches after
a 0.5 s warm-up; the labels of the last launch are saved and compared with the
first build's (count of differing windows).  AB_ARITH=f32 times the
exact-f32 kernel instead of the split-f16 one."""
import json
import os
import subprocess
import sys

import numpy as np

CHILD = r'''
import json, os, sys, time, torch, numpy as np
sys.path.insert(0, os.getcwd())
from bench import synth_audio
from vad_amd.ffn import TOPOLOGY_BL13, TOPOLOGY_REF39, FFNClassifier, random_layers
from vad_amd.pipeline import VadPipeline
dev = torch.device("cuda", 0)
F = 1_000_000
a = synth_audio(160 * (F - 1) + 401, 1, dev)
m = VadPipeline().mfcc(a)
out = {}
for name, topo in (("bl13", TOPOLOGY_BL13), ("ref39", TOPOLOGY_REF39)):
    plan = FFNClassifier(random_layers(topo, seed=3), arith=os.environ.get("AB_ARITH", "split_f16")).plan
    lab = torch.empty((F - 5,), dtype=torch.uint8, device=dev)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.5:
        plan.window_labels(m, out=lab)
    torch.cuda.synchronize()
    ts = []
    for _ in range(7):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(20):
            plan.window_labels(m, out=lab)
        e.record(); torch.cuda.synchronize()
        ts.append(s.elapsed_time(e) / 20 * 1e3)
    ts.sort()
    out[name + "_us"] = ts[3]
    np.save(os.environ["AB_OUT"] + f"_{name}.npy", lab.cpu().numpy())
print(json.dumps(out))
'''

args = sys.argv[1:]
rounds = int(args.pop()) if args and args[-1].isdigit() else 3
os.makedirs("gpurun_out", exist_ok=True)
res = {l: [] for l in args}
for r in range(rounds):
    for i, l in enumerate(args):
        env = dict(os.environ, VAD_AMD_LIB=l, AB_OUT=f"gpurun_out/abffn_{i}")
        p = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
        line = [x for x in p.stdout.splitlines() if x.startswith("{")]
        res[l].append(json.loads(line[-1]) if line else {"error": p.stderr[-400:]})
summary = {}
for i, l in enumerate(args):
    d = {}
    for k in ("bl13_us", "ref39_us"):
        xs = sorted(x[k] for x in res[l] if k in x)
        d[k] = xs[len(xs) // 2] if xs else None
        d[k + "_all"] = [round(x, 2) for x in xs]
    for name in ("bl13", "ref39"):
        a = np.load(f"gpurun_out/abffn_0_{name}.npy")
        b = np.load(f"gpurun_out/abffn_{i}_{name}.npy")
        d[name + "_labels_differ_from_first"] = int((a != b).sum())
    summary[os.path.basename(l)] = d
print(json.dumps(summary))
