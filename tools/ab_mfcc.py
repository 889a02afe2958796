"""A/B of MFCC kernel builds on one box: python tools/ab_mfcc.py LIB_A LIB_B [LIB_C ...] [rounds]
Alternates the two libraries (fresh processes) and prints per-launch us for
C3 (1M frames) and C2 (100k, 6 rotated clips), fp32 input (int16 PCM with AB_I16=1)."""
import json
import os
import subprocess
import sys

CHILD = r'''
import json, os, sys, torch
sys.path.insert(0, os.getcwd())
from bench import synth_audio
from vad_amd.pipeline import VadPipeline
dev = torch.device("cuda", 0)
pipe = VadPipeline()
def t(fn, reps=100, warm=200):
    for _ in range(warm): fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(); s.record()
    for _ in range(reps): fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3
F = 1_000_000
a = synth_audio(160 * (F - 1) + 401, 1, dev); m = torch.empty((F, 13), device=dev)
if os.environ.get("AB_I16"): a = a.to(torch.int16)
c3 = t(lambda: pipe.mfcc(a, out=m))
del a, m
F = 100_000
cl = [synth_audio(160 * (F - 1) + 401, 10 + i, dev) for i in range(6)]; m = torch.empty((F, 13), device=dev)
if os.environ.get("AB_I16"): cl = [c.to(torch.int16) for c in cl]
k = [0]
def c2f():
    pipe.mfcc(cl[k[0] % 6], out=m); k[0] += 1
c2 = t(c2f)
from vad_amd.config import MfccConfig
p40 = VadPipeline(cfg=MfccConfig(n_filters=40))
def c2g():
    p40.mfcc(cl[k[0] % 6], out=m); k[0] += 1
c2_40 = t(c2g)
print(json.dumps({"c3_us": c3, "c2_us": c2, "c2_40_us": c2_40}))
'''

args = sys.argv[1:]
rounds = int(args.pop()) if args and args[-1].isdigit() else 3
libs = args
res = {l: [] for l in libs}
for r in range(rounds):
    for l in libs:
        env = dict(os.environ, VAD_AMD_LIB=l)
        out = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=120)
        line = [x for x in out.stdout.splitlines() if x.startswith("{")]
        res[l].append(json.loads(line[-1]) if line else {"error": out.stderr[-300:]})
print(json.dumps(res))
