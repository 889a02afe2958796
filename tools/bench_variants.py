"""Secondary measurements beside bench.py's headline line:

  C2   MFCC only, 100k frames (fp32 input)               frames/s, kernel us
  C3m  MFCC only, 1M frames, fp32 vs int16 PCM input      frames/s, kernel us
  C3f  MFCC + FFN, 1M frames, ref39 vs bl13               frames/s
  C5   512 analyser streams, one hop per step, hipGraph   us per hop (all streams)
  tree / SimpleAnalyser feature kernels                   kernel us

Kernel times are HIP events on the launching stream around N repeats after
warm-up; inputs are device-resident.  Prints one JSON object.

    python tools/bench_variants.py [--reps 50]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import synth_audio  # noqa: E402
from vad_amd import ffn as ffn_mod  # noqa: E402
from vad_amd.pipeline import VadPipeline  # noqa: E402
from vad_amd.stream import StreamBatch  # noqa: E402


def timed(fn, reps, warm=100):  # warm-up past a cold GPU's clock ramp
    for _ in range(warm):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e-3  # seconds per call


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    dev = torch.device("cuda")
    res = {}
    pipe = VadPipeline()

    # C2: 100k frames, fp32
    F = 100_000
    x = synth_audio(160 * (F - 1) + 401, 0, dev)
    out = torch.empty((F, 13), device=dev)
    t = timed(lambda: pipe.mfcc(x, out=out), a.reps)
    res["C2_mfcc_100k"] = {"frames_per_s": F / t, "us": t * 1e6}
    # BASELINE configs[1] names 40 mel filters
    from vad_amd.config import MfccConfig
    pipe40 = VadPipeline(cfg=MfccConfig(n_filters=40))
    t = timed(lambda: pipe40.mfcc(x, out=out), a.reps)
    res["C2_mfcc_100k_40mel"] = {"frames_per_s": F / t, "us": t * 1e6}

    # MFCC only at 1M frames: fp32 vs int16 input
    F = 1_000_000
    x = synth_audio(160 * (F - 1) + 401, 1, dev)
    x16 = x.to(torch.int16)
    out = torch.empty((F, 13), device=dev)
    t32 = timed(lambda: pipe.mfcc(x, out=out), a.reps)
    t16 = timed(lambda: pipe.mfcc(x16, out=out), a.reps)
    res["C3_mfcc_1M_fp32"] = {"frames_per_s": F / t32, "us": t32 * 1e6,
                              "GBps_algorithmic": 692 * F / t32 / 1e9}
    res["C3_mfcc_1M_int16"] = {"frames_per_s": F / t16, "us": t16 * 1e6,
                               "GBps_algorithmic": (320 + 52) * F / t16 / 1e9}

    # MFCC + FFN, both compiled topologies
    for name, topo in (("bl13", ffn_mod.TOPOLOGY_BL13), ("ref39", ffn_mod.TOPOLOGY_REF39)):
        clf = ffn_mod.FFNClassifier(ffn_mod.random_layers(topo, seed=3))
        p = VadPipeline(ffn=clf)
        lab = torch.empty((F - 5,), dtype=torch.uint8, device=dev)

        def step():
            m = p.mfcc(x, out=out)
            clf.plan.window_labels(m, out=lab)
        t = timed(step, max(10, a.reps // 2))
        res[f"C3_mfcc_ffn_{name}"] = {"frames_per_s": F / t, "us": t * 1e6}

    # PCIe-inclusive: the clip in pinned host memory (fp32, and int16 PCM at
    # half the bytes) -> H2D copy -> fused MFCC + features + FFN -> labels
    clf = ffn_mod.FFNClassifier(ffn_mod.random_layers(ffn_mod.TOPOLOGY_BL13, seed=3))
    p = VadPipeline(ffn=clf)
    lab = torch.empty((F - 5,), dtype=torch.uint8, device=dev)
    for name, src in (("fp32", x), ("int16", x16)):
        host = src.cpu().pin_memory()
        dbuf = torch.empty_like(src)

        def e2e():
            dbuf.copy_(host, non_blocking=True)
            p.labels(dbuf, out=lab)
        t = timed(e2e, max(10, a.reps // 2), warm=10)
        res[f"C3_host_clip_to_labels_{name}"] = {"frames_per_s": F / t, "us": t * 1e6,
                                                 "host_bytes": host.numel() * host.element_size()}

    # MFCC + decision tree (the classifier vad.py deploys), fixture tree
    from vad_amd.tree import TreeClassifier
    gt = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests",
                      "golden", "tree.npz")
    with __import__("numpy").load(gt, allow_pickle=False) as g:
        tree = TreeClassifier(g["feature"], g["threshold"], g["left"], g["right"], g["leaf"],
                              g["nan_left"], g["classes"], int(g["n_features"]))
    lab = torch.empty((F - 5,), dtype=torch.uint8, device=dev)

    def step_tree():
        m = pipe.mfcc(x, out=out)
        tree.window_labels(m, out=lab)
    t = timed(step_tree, max(10, a.reps // 2))
    tt = timed(lambda: tree.window_labels(out, out=lab), max(10, a.reps // 2))
    res["C3_mfcc_tree"] = {"frames_per_s": F / t, "us": t * 1e6, "tree_kernel_us": tt * 1e6,
                           "nodes": int(len(tree.feature))}

    # SimpleAnalyser per-frame features (fp64: stEnergy, stZCR, std|fft|, 4 bands),
    # 100k frames of 400 samples (fft 512), one launch
    from vad_amd import _lib
    from vad_amd.simple_analyser import SimpleAnalyser
    sa = SimpleAnalyser(16000, 400, 10)
    Fs = 100_000
    fr = x[: 160 * (Fs - 1) + 400].unfold(0, 400, 160).contiguous()
    sf = torch.empty((Fs, 7), dtype=torch.float64, device=dev)
    lib = _lib.lib()

    def simple():
        _lib.check(lib.vad_simple_features(_lib.ptr(fr), Fs, 400, 400, sa._fft_len(),
                                           sa.fft_extended_zeros, sa.fftn_for_band, 4, _lib.ptr(sf),
                                           _lib.stream_ptr()), "vad_simple_features")
    t = timed(simple, a.reps)
    res["simple_features_100k"] = {"frames_per_s": Fs / t, "us": t * 1e6}

    # C5: 512 streams, one 10 ms hop per step, replayed hipGraph
    S = 512
    clf = ffn_mod.FFNClassifier(ffn_mod.random_layers(ffn_mod.TOPOLOGY_BL13, seed=3))
    sb = StreamBatch(S, clf)
    g = torch.Generator(device=dev).manual_seed(500)
    sb.prime(torch.randn((S, 240), generator=g, device=dev) * 1000)
    hops = [torch.randn((S, 160), generator=g, device=dev) * 1000 for _ in range(8)]
    sb.capture()
    k = [0]

    def hop():
        sb.step(hops[k[0] % 8])
        k[0] += 1
    t = timed(hop, max(100, a.reps * 4))
    res["C5_stream_512"] = {"us_per_hop": t * 1e6, "stream_frames_per_s": S / t,
                            "realtime_factor": 0.010 / t}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
