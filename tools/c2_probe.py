"""C2 (100k frames, MFCC only) timing probe: HIP events around back-to-back
launches vs the host time per call (is the launch rate host-bound?), and a
hipGraph of the same launches.  python tools/c2_probe.py [reps]"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import synth_audio  # noqa: E402
from vad_amd.config import MfccConfig  # noqa: E402
from vad_amd.pipeline import VadPipeline  # noqa: E402

dev = torch.device("cuda", 0)
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 60
F = 100_000
clips = [synth_audio(160 * (F - 1) + 401, 10 + i, dev) for i in range(6)]
mf = torch.empty((F, 13), dtype=torch.float32, device=dev)
res = {}
for nf in (40, 26):
    pipe = VadPipeline(cfg=MfccConfig(n_filters=nf))
    for k in range(60):
        pipe.mfcc(clips[k % 6], out=mf)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    s.record()
    for k in range(reps):
        pipe.mfcc(clips[k % 6], out=mf)
    e.record()
    t_host = (time.perf_counter() - t0) / reps
    torch.cuda.synchronize()
    ev = s.elapsed_time(e) / reps * 1e3
    # the same launches captured once into a graph
    g = torch.cuda.CUDAGraph()
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(st):
        pipe.mfcc(clips[0], out=mf)
    torch.cuda.current_stream().wait_stream(st)
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        for k in range(12):
            pipe.mfcc(clips[k % 6], out=mf)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps // 12):
        g.replay()
    e.record()
    torch.cuda.synchronize()
    gr = s.elapsed_time(e) / ((reps // 12) * 12) * 1e3
    res[nf] = {"events_us": ev, "host_us_per_call": t_host * 1e6, "graph_us": gr}
print(json.dumps(res))
