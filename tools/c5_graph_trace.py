"""C5 one-hop step, direct launch vs hipGraph replay, for a rocprofv3 trace
(verdict r05: where do the one-hop graph replay's extra ~5 us go?):
    rocprofv3 --kernel-trace --hip-runtime-trace --stats -d gpurun_out/c5g -- python3 tools/c5_graph_trace.py
Phases (each N back-to-back steps of 512 streams, 13-64-64-2, device input):
direct one-hop launches, one-hop graph replays (vad_graph_plan_launch: the
capture's single kernel node dispatched directly), and the same replays
through hipGraphLaunch (vad_graph_launch).
Prints host-clock and event us per hop for each phase."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vad_amd import ffn as ffn_mod  # noqa: E402
from vad_amd.stream import StreamBatch  # noqa: E402

S, N = 512, int(os.environ.get("C5_STEPS", "400"))
dev = torch.device("cuda")
clf = ffn_mod.FFNClassifier(ffn_mod.random_layers(ffn_mod.TOPOLOGY_BL13, seed=3))
out = {}
import ctypes  # noqa: E402
from vad_amd import _lib  # noqa: E402

for name, graph in (("direct", False), ("graph", True), ("graph_hipGraphLaunch", "raw"),
                    ("direct2", False), ("graph2", True), ("graph_hipGraphLaunch2", "raw")):
    sb = StreamBatch(S, clf)
    g = torch.Generator(device=dev).manual_seed(500)
    sb.prime(torch.randn((S, 240), generator=g, device=dev) * 1000)
    sb.inputs.copy_(torch.randn((1, S, 160), generator=g, device=dev) * 1000)
    if graph:
        sb.capture()
    if graph == "raw":  # every replay through hipGraphLaunch (vad_graph_launch)
        ex, lib = ctypes.c_void_p(sb.graph.raw_cuda_graph_exec()), _lib.lib()
        step = lambda: lib.vad_graph_launch(ex, _lib.stream_ptr())  # noqa: E731
    else:
        step = sb.step_block if graph else (lambda: sb.step(sb.hop_in))
    for _ in range(200):
        step()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    s.record()
    for _ in range(N):
        step()
    e.record()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    out[name] = {"graph_direct": sb.graph_direct, "event_us_per_hop": s.elapsed_time(e) / N * 1e3,
                 "host_issue_us_per_hop": (t1 - t0) / N * 1e6, "host_total_us_per_hop": (t2 - t0) / N * 1e6}
print(json.dumps(out))
