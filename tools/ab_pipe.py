"""A/B of pipelined C3 steps across library builds, fresh processes
alternated: python tools/ab_pipe.py LIB_A LIB_B [...] [rounds]

Per build and round: 1M-frame clip, 13-64-64-2; consecutive steps (MFCC
kernel + FFN kernel, vad_mfcc_ffn with a workspace) alternate over two HIP
streams as in bench.py, so a step's FFN can run beside the next step's MFCC;
also the same steps serial on one stream.  Median of 5 batches of 200 steps
after 600 warm-up steps."""
import json
import os
import statistics
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
s0 = torch.cuda.current_stream(); s1 = torch.cuda.Stream(device=dev); s1.wait_stream(s0)
labs = [torch.empty((F - 5,), dtype=torch.uint8, device=dev) for _ in range(2)]
streams = [s0, s1]
def run(n, two):
    for i in range(n):
        k = i % 2 if two else 0
        with torch.cuda.stream(streams[k]):
            pipe.labels(a, out=labs[k])
def timed(two, n=200):
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s0)
    run(n, two)
    s0.wait_stream(s1)
    e1.record(s0)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3
run(600, True)
out = {"pipe_us": sorted(timed(True) for _ in range(5))[2], "serial_us": sorted(timed(False) for _ in range(5))[2]}
out["labels_sum"] = int(labs[0].sum()); out["labels_equal"] = bool(torch.equal(labs[0], labs[1]))
print(json.dumps(out))
'''

args = sys.argv[1:]
rounds = int(args.pop()) if args and args[-1].isdigit() else 3
res = {l: [] for l in args}
for r in range(rounds):
    for lib in args:
        env = dict(os.environ, VAD_AMD_LIB=lib)
        p = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
        if p.returncode != 0:
            sys.stderr.write(p.stderr)
            sys.exit(p.returncode)
        res[lib].append(json.loads(p.stdout.strip().splitlines()[-1]))
        print(lib, res[lib][-1], file=sys.stderr, flush=True)
summary = {}
for lib, rs in res.items():
    summary[os.path.basename(lib)] = {
        "pipe_us": statistics.median(x["pipe_us"] for x in rs),
        "pipe_us_all": sorted(round(x["pipe_us"], 2) for x in rs),
        "serial_us": statistics.median(x["serial_us"] for x in rs),
        "serial_us_all": sorted(round(x["serial_us"], 2) for x in rs),
        "labels_sum": sorted({x["labels_sum"] for x in rs}),
        "labels_equal": all(x["labels_equal"] for x in rs)}
print(json.dumps(summary))
