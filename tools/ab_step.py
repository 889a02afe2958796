"""A/B of whole C3 steps (vad_mfcc_ffn with a workspace: MFCC kernel + FFN
kernel, 1M frames, 13-64-64-2) across library builds, fresh processes
alternated: python tools/ab_step.py LIB_A LIB_B [...] [rounds]"""
import json
import os
import subprocess
import sys

CHILD = r'''
import json, os, sys, torch
sys.path.insert(0, os.getcwd())
from bench import synth_audio
from vad_amd.ffn import TOPOLOGY_BL13, FFNClassifier, random_layers
from vad_amd.pipeline import VadPipeline
dev = torch.device("cuda", 0)
pipe = VadPipeline(FFNClassifier(random_layers(TOPOLOGY_BL13, seed=3)))
F = 1_000_000
a = synth_audio(160 * (F - 1) + 401, 1, dev)
lab = torch.empty((F - 5,), dtype=torch.uint8, device=dev)
for _ in range(300): pipe.labels(a, out=lab)
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
torch.cuda.synchronize(); s.record()
for _ in range(200): pipe.labels(a, out=lab)
e.record(); torch.cuda.synchronize()
print(json.dumps({"step_us": s.elapsed_time(e) / 200 * 1e3, "labels_sum": int(lab.sum())}))
'''

args = sys.argv[1:]
rounds = int(args.pop()) if args and args[-1].isdigit() else 3
res = {l: [] for l in args}
for r in range(rounds):
    for l in args:
        env = dict(os.environ, VAD_AMD_LIB=l)
        out = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=180)
        line = [x for x in out.stdout.splitlines() if x.startswith("{")]
        res[l].append(json.loads(line[-1]) if line else {"error": out.stderr[-300:]})
print(json.dumps(res))
for l, v in res.items():
    xs = sorted(x.get("step_us", 0) for x in v)
    print(f"{os.path.basename(l):28s} step {xs[len(xs) // 2]:7.1f} us  {[round(x, 1) for x in xs]}")
