"""Benchmark: MFCC+FFN frames/s on synthetic 16 kHz audio (BASELINE.json).

Workload (one step, per rank): one clip of F = 1,000,000 frames of 25 ms at a
10 ms hop (160*(F-1)+401 fp32 samples, already resident in HBM), framed ->
MFCC (HIP kernel) -> 5-frame analyser features + FFN on split-f16 MFMA (HIP
kernel) -> F-5 uint8 labels; with N > 1 ranks each rank classifies its own
clip (weak scaling, no data-path collective) and the per-window decisions are
gathered to rank 0 over RCCL inside the step (BASELINE configs 3 and 4).
Consecutive steps alternate over --streams HIP streams (default 2, each with
its own workspace and label buffer): step k + 1's MFCC kernel starts on the
CUs that step k's MFCC tail and FFN leave idle; every step still runs its
whole clip through both kernels inside the timed region.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--frames F] [--ffn bl13|ref39] [--streams S]

Rank 0 prints ONE JSON line.  `value` = frames (MFCC frames) processed by all
ranks / max-over-ranks wall time of the K timed steps.  `roofline` is for the
dominant kernel (the MFCC kernel): its average launch duration comes from HIP
events on the stream it is launched on, around K back-to-back launches right
after the timed region (events between the step's kernels would idle the GPU
~5 us each, so the timed steps carry none); `cpu_baseline` times the oracle's vectorised NumPy restatement
on a bounded sample on one host core (rank 0, N = 1 only), and
`cpu_baseline_all_cores` the same loop on up to 16 cores, one process each.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec
HBM_COPY_GBS = 6290.0          # MI355X_MICROARCH.md: measured device copy (SURVEY 8(d) asks for both)
MFCC_BYTES_PER_FRAME = 160 * 4 + 13 * 4   # new samples in + 13 fp32 out
FFN_BYTES_PER_FRAME = 13 * 4 + 1          # MFCC row in + uint8 label out
# SURVEY 8(d) algorithmic flops per frame of the MFCC kernel: FFT 11,520 +
# power 768 + sparse mel 888 + log 26 + lifter x DCT 676
MFCC_FLOPS_PER_FRAME = 13878
VALU_PEAK_TFS = 157.3          # MI355X_MICROARCH.md: peak FP32 (vector)
# The MFCC kernel's VALU issue model ("Where the ceiling
# is"): packed / scalar VALU wave-instructions per frame from its ISA and PMC
# (profiles/r02b_pmc.txt: 93.1 in all), and the per-SIMD cost of one at two
# waves per SIMD measured on this part (profiles/r02_valu_rates.txt)
MFCC_VALU_PACKED_PER_FRAME = 60
MFCC_VALU_SCALAR_PER_FRAME = 33
VALU_NS_PACKED_2W = 3.02
VALU_NS_SCALAR_2W = 1.51
N_SIMDS = 1024                 # 256 CUs x 4


def synth_audio(n_samples, seed, device):
    """int16-range noise with per-1600-sample amplitude 10**U(0,4), 5% silent
    segments; generated on the device."""
    g = torch.Generator(device=device).manual_seed(seed)
    seg = 1600
    n_seg = (n_samples + seg - 1) // seg
    amp = 10.0 ** (torch.rand(n_seg, generator=g, device=device) * 4.0)
    amp[torch.rand(n_seg, generator=g, device=device) < 0.05] = 0.0
    x = torch.randn(n_seg * seg, generator=g, device=device) * amp.repeat_interleave(seg)
    return x[:n_samples].round_().clamp_(-32767, 32767).contiguous()


def cpu_baseline(layers, frames_per_chunk=20000, min_seconds=10.0, max_chunks=100):
    """Oracle (NumPy restatement, test infrastructure) on one core, bounded sample."""
    try:
        from threadpoolctl import threadpool_limits
    except ImportError:  # pragma: no cover
        threadpool_limits = None
    from oracle import vad_oracle as O
    fb = O.get_mel_filterbanks(300, 8000, 512, 26, 16000)
    clip = O.synth_clip(160 * (frames_per_chunk - 1) + 401, seed=1)
    ctx = threadpool_limits(limits=1) if threadpool_limits else None
    if ctx:
        ctx.__enter__()
    try:
        n, t0 = 0, time.perf_counter()
        while True:
            m = O.mfcc_batch(clip, fb)
            x = O.analyser_features_fast(m)
            O.ffn_labels(x[:, :layers[0][0].shape[0]], layers)
            n += len(m)
            el = time.perf_counter() - t0
            if el >= min_seconds or n >= frames_per_chunk * max_chunks:
                break
    finally:
        if ctx:
            ctx.__exit__(None, None, None)
    return {"value": n / el, "unit": "frames/s", "cores": 1, "kind": "port",
            "sample": f"{n} frames ({n // frames_per_chunk} x {frames_per_chunk}-frame synthetic "
                      f"clips), oracle/vad_oracle.py vectorised NumPy (pocketfft f32 FFT, fp64 "
                      f"mel/log/DCT, fp64 features + FFN), {el:.1f} s"}


def _cpu_chunks(args):
    """Worker of cpu_baseline_all: the same per-chunk oracle loop on one core."""
    n_in, frames_per_chunk, seconds, dims = args
    from threadpoolctl import threadpool_limits
    from oracle import vad_oracle as O
    from vad_amd.ffn import random_layers
    layers = random_layers(dims, seed=3)
    fb = O.get_mel_filterbanks(300, 8000, 512, 26, 16000)
    clip = O.synth_clip(160 * (frames_per_chunk - 1) + 401, seed=1)
    with threadpool_limits(limits=1):
        n, t0 = 0, time.perf_counter()
        while n < n_in and time.perf_counter() - t0 < seconds:
            m = O.mfcc_batch(clip, fb)
            x = O.analyser_features_fast(m)
            O.ffn_labels(x[:, :dims[0]], layers)
            n += len(m)
    return n


def _cpu_per_frame(args):
    """Reference-shaped loop (variant (i) of SURVEY 8(d)): per frame
    mfcc.get_mfcc (np.fft.fft -> dot -> log10 -> dct -> lifter, mfcc.py:67-78)
    into a 5-frame buffer, per window the analyser's (1, 39) feature row and
    a batch-1 FFN predict (sklearn_analyser.py:52-71) -- the oracle's
    per-frame functions, one core.  Returns frames done in `seconds`."""
    seconds, dims = args
    from threadpoolctl import threadpool_limits
    from oracle import vad_oracle as O
    from vad_amd.ffn import random_layers
    layers = random_layers(dims, seed=3)
    fb = O.get_mel_filterbanks(300, 8000, 512, 26, 16000)
    clip = O.synth_clip(160 * 20000 + 241, seed=1)
    fr = O.frame_matrix(clip)
    with threadpool_limits(limits=1):
        buf, n, t0 = [], 0, time.perf_counter()
        while time.perf_counter() - t0 < seconds:
            buf.append(O.get_mfcc(fr[n % len(fr)], 512, fb, 13))
            if len(buf) > 5:
                buf.pop(0)
            if len(buf) == 5:
                x = O.window_features(np.stack(buf))[None, :dims[0]]
                O.ffn_labels(x, layers)
            n += 1
    return n


def host_facts():
    """CPU model, cores this process may use, NumPy / SciPy versions."""
    import scipy
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"cpu_model": model, "cores_available": len(os.sched_getaffinity(0)),
            "numpy": np.__version__, "scipy": scipy.__version__}


def cpu_baseline_per_frame(dims, seconds=5.0):
    """Variant (i): the reference-shaped per-frame loop on 1 core and on up to
    16 cores (one spawned process each, like dataset_creator.py:84's Pool)."""
    import multiprocessing as mp
    n1 = _cpu_per_frame((seconds, tuple(dims)))
    one = {"value": n1 / seconds, "unit": "frames/s", "cores": 1, "kind": "port",
           "sample": f"{n1} frames, per-frame get_mfcc + per-window features + batch-1 FFN, {seconds:.0f} s"}
    n_proc = max(1, min(16, len(os.sched_getaffinity(0))))
    ctx = mp.get_context("spawn")
    with ctx.Pool(n_proc) as pool:
        pool.map(_cpu_per_frame, [(0.5, tuple(dims))] * n_proc)  # imports, warm caches
        t0 = time.perf_counter()
        n = sum(pool.map(_cpu_per_frame, [(seconds, tuple(dims))] * n_proc))
        el = time.perf_counter() - t0
    allc = {"value": n / el, "unit": "frames/s", "cores": n_proc, "kind": "port",
            "sample": f"{n} frames on {n_proc} processes x 1 thread, same per-frame loop, {el:.1f} s"}
    return one, allc


def cpu_baseline_all(dims, frames_per_chunk=20000, seconds=6.0):
    """The same oracle loop on every host core this process may use (at most
    16, the GPU box's CPU share), one process per core (spawned: no fork of
    the GPU process), like dataset_creator.py's multiprocessing pool."""
    import multiprocessing as mp
    n_proc = max(1, min(16, len(os.sched_getaffinity(0))))
    ctx = mp.get_context("spawn")
    with ctx.Pool(n_proc) as pool:
        pool.map(_cpu_chunks, [(frames_per_chunk, frames_per_chunk, 60.0, dims)] * n_proc)  # warm
        t0 = time.perf_counter()
        n = sum(pool.map(_cpu_chunks, [(10 ** 9, frames_per_chunk, seconds, dims)] * n_proc))
        el = time.perf_counter() - t0
    return {"value": n / el, "unit": "frames/s", "cores": n_proc, "kind": "port",
            "sample": f"{n} frames on {n_proc} processes x 1 thread, same loop as cpu_baseline, "
                      f"{el:.1f} s"}


def feed_frame_latency(dev, calls=2000, warm=50):
    """Per-call latency of the drop-in SKLearnAnalyzer.feed_frame (the API
    vad.py:52 calls once per 25 ms block): one 400-sample frame in, the
    frame three calls back or None out -- H2D copy, the MFCC + features + FFN
    kernels on the stream's device state, the label read back.  A 2-class
    39-64-32-16-2 network (labels 0/1 only, as vad.py's dispatch expects)."""
    import tempfile
    from oracle import vad_oracle as O
    from vad_amd.ffn import random_layers, save_layers
    from vad_amd.sklearn_analyser import SKLearnAnalyzer
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "ffn.npz")
        save_layers(path, random_layers((39, 64, 32, 16, 2), seed=3))
        an = SKLearnAnalyzer(path)
    clip = O.synth_clip(400 * (calls + warm + 5), seed=2).reshape(-1, 400)
    an.load_init_inactive_frames(list(clip[:5]))
    frames = list(clip[5:])
    for f in frames[:warm]:
        an.feed_frame(f)
    per = []
    for f in frames[warm:warm + calls]:
        t0 = time.perf_counter()
        an.feed_frame(f)
        per.append(time.perf_counter() - t0)
    per = np.sort(np.asarray(per)) * 1e3
    return {"ms_per_call_mean": float(per.mean()), "p50": float(per[len(per) // 2]),
            "p99": float(per[int(0.99 * len(per))]), "calls": calls,
            "reference_ms_per_call": 3.07,
            "reference_source": "SURVEY.md section 6: SKLearnAnalyzer.feed_frame on this container's CPU "
                                "(not re-measured here: the reference cannot travel to the GPU box)"}


def secondary_configs(dev, reps=60):
    """The other BASELINE configs beside the headline (rank 0, N = 1):
    C2 (configs[1]) MFCC only, 100k frames, 40 and 26 mel: six clips rotated
    per launch (384 MB, past the 256 MiB Infinity Cache), HIP events around
    `reps` launches; C5 (configs[4]) 512 analyser streams, one 10 ms hop per
    step: the single-kernel hop and the three-kernel hipGraph replay."""
    from vad_amd.config import MfccConfig
    from vad_amd.ffn import TOPOLOGY_BL13, FFNClassifier, random_layers
    from vad_amd.pipeline import VadPipeline
    from vad_amd.stream import StreamBatch
    out = {}
    F = 100_000
    clips = [synth_audio(160 * (F - 1) + 401, 10 + i, dev) for i in range(6)]
    mf = torch.empty((F, 13), dtype=torch.float32, device=dev)
    for nf in (40, 26):
        pipe = VadPipeline(cfg=MfccConfig(n_filters=nf))
        # warm up by time, as the headline does: this runs after the latency
        # loop, whose tiny kernels leave the GPU clock low (60 launches = 2 ms
        # measured the clock ramp: 39 vs 33 us at 40 mel)
        t_end = time.perf_counter() + 0.3
        k = 0
        while time.perf_counter() < t_end or k < 60:
            pipe.mfcc(clips[k % 6], out=mf)
            k += 1
            if k % 60 == 0:
                torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        s.record()
        for k in range(reps):
            pipe.mfcc(clips[k % 6], out=mf)
        e.record()
        torch.cuda.synchronize()
        t = s.elapsed_time(e) / reps * 1e-3
        # the same launches alternating over two streams (own output buffers):
        # a batch's launch ramp and tail overlap its neighbours' -- the
        # throughput of a stream of 100k-frame batches, not a launch time
        cur = torch.cuda.current_stream()
        st2 = [cur, torch.cuda.Stream(device=dev)]
        mf2 = [mf, torch.empty_like(mf)]
        st2[1].wait_stream(cur)
        torch.cuda.synchronize()
        s.record(cur)
        for k in range(reps):
            with torch.cuda.stream(st2[k % 2]):
                pipe.mfcc(clips[k % 6], out=mf2[k % 2])
        cur.wait_stream(st2[1])
        e.record(cur)
        torch.cuda.synchronize()
        tp = s.elapsed_time(e) / reps * 1e-3
        out[f"c2_mfcc_100k_{nf}mel"] = {
            "frames_per_s": F / t, "avg_launch_us": t * 1e6,
            "achieved_GBps": MFCC_BYTES_PER_FRAME * F / t / 1e9,
            "frac_hbm": MFCC_BYTES_PER_FRAME * F / t / 1e9 / HBM_PEAK_GBS,
            "pipelined_us_per_batch": tp * 1e6,
            "pipelined_frac_hbm": MFCC_BYTES_PER_FRAME * F / tp / 1e9 / HBM_PEAK_GBS,
            "note": "6 rotated 64 MB clips (384 MB working set); avg_launch_us: back-to-back launches on "
                    "one stream; pipelined_us_per_batch: the same launches alternating over two streams"}
    del clips
    S = 512
    # BASELINE configs[4]: 512 streams, hipGraph-captured hops.  Device-input
    # lines (the hop block already in HBM): the one-kernel hop launched
    # directly (input read in place); K = 8 hops per replay of a graph that
    # reads its static block in place (hop_kernel_hipgraph: the round-3
    # meaning of that key, kept across rounds); one hop per replay, in place
    # and with an eager copy into the static block before each replay
    # (_1hop, _1hop_with_copy); K = 8 hops per direct launch
    # (vad_stream_hops: tables staged once per launch, stream state carried
    # in registers); the three-kernel form captured.  End-to-end lines (C5's rate includes the H2D
    # copy): each step copies the 512 x 160 new samples of its K hops from
    # pinned host memory, runs the hop kernel and copies the K x 512 labels
    # back (StreamBatch.step_host), launched directly or as ONE graph replay
    # (vad_graph_plan_launch) -- us_per_hop back to back, and latency_us = one
    # step until its labels are in host memory (stream sync, host clock).
    clf = FFNClassifier(random_layers(TOPOLOGY_BL13, seed=3))
    for name, kernel, K, graph, copy, host in (
            ("hop_kernel", "hop", 1, False, False, False),
            ("hop_kernel_hipgraph", "hop", 8, True, False, False),
            ("hop_kernel_hipgraph_1hop", "hop", 1, True, False, False),
            ("hop_kernel_hipgraph_1hop_with_copy", "hop", 1, True, True, False),
            ("hop_kernel_x8", "hop", 8, False, False, False),
            ("three_kernel_hipgraph", "three", 1, True, True, False),
            ("e2e_host_io_direct", "hop", 1, False, False, True),
            ("e2e_host_io_hipgraph", "hop", 1, True, False, True),
            ("e2e_host_io_direct_x8", "hop", 8, False, False, True),
            ("e2e_host_io_hipgraph_x8", "hop", 8, True, False, True)):
        sb = StreamBatch(S, clf, kernel=kernel, hops_per_step=K)
        g = torch.Generator(device=dev).manual_seed(500)
        sb.prime(torch.randn((S, 240), generator=g, device=dev) * 1000)
        blocks = [torch.randn((K, S, 160), generator=g, device=dev) * 1000 for _ in range(8)]
        sb.inputs.copy_(blocks[0])
        if host:
            sb.attach_host_io()
            sb.host_inputs.copy_(blocks[0].cpu())
        if graph:
            sb.capture(host_io=host)

        def one(k):
            if host:
                sb.step_host()  # the producer writes host_inputs between steps
            elif graph and not copy:
                sb.step_block()  # the static block, written in place by the producer
            elif K == 1:
                sb.step(blocks[k % 8][0])
            else:
                sb.step_block(blocks[k % 8])

        reps = max(50, 400 // K)
        for k in range(max(25, 200 // K)):
            one(k)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        s.record()
        for k in range(reps):
            one(k)
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) / (reps * K) * 1e3
        rec = {"us_per_hop": us, "stream_frames_per_s": S / (us * 1e-6),
               "x_real_time": 10_000.0 / us, "hops_per_launch_or_replay": K,
               "hipgraph": graph, "input_copy_per_step": copy or host,
               "host_io": host}
        if host:
            cur = torch.cuda.current_stream()
            lat = []
            for k in range(200):
                t0 = time.perf_counter()
                one(k)
                cur.synchronize()
                lat.append(time.perf_counter() - t0)
            lat = np.sort(np.asarray(lat)) * 1e6
            rec["bytes_per_step"] = {"h2d": K * S * 160 * 4, "d2h": K * S}
            rec["latency_us"] = {"p50": float(lat[len(lat) // 2]), "p90": float(lat[int(0.9 * len(lat))]),
                                 "mean": float(lat.mean())}
        out[f"c5_512_streams_{name}"] = rec
    return out


def launch_ranks(n):
    """Run this script as n ranks under torch.distributed.run (127.0.0.1, a
    free port); called before any GPU call of the parent process, which only
    waits for the children (no exec)."""
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=30)  # past the clock ramp of a cold GPU
    ap.add_argument("--frames", type=int, default=1_000_000)
    ap.add_argument("--ffn", default="bl13", choices=["bl13", "ref39"])
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-secondary", action="store_true")  # skip the C2 / C5 lines (profiling runs)
    # gloo: rehearse the N > 1 path on fewer GPUs than ranks (ranks share
    # devices round-robin; the labels travel through host memory)
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"])
    # a GPU that was idle starts at low clocks and ramps for ~30 ms of load:
    # warm-up steps continue (untimed) until this much warm-up time has passed
    ap.add_argument("--min-warmup-s", type=float, default=0.5)
    # consecutive clips alternate over this many HIP streams (each with its
    # own MFCC workspace and label buffer), so clip k + 1's MFCC fills the
    # CUs that clip k's MFCC tail and FFN leave idle; 1 = strictly serial
    ap.add_argument("--streams", type=int, default=2)
    args = ap.parse_args()
    if args.streams < 1:
        ap.error("--streams must be >= 1")
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")

    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        # --gpus N without a launcher: start N rank processes (one per GPU)
        # under torch.distributed.run before this process touches the GPU,
        # and exit with their status (rank 0 prints the JSON line)
        sys.exit(launch_ranks(args.gpus))
    if env_world is not None and int(env_world) != args.gpus:
        print(f"bench.py: --gpus {args.gpus} disagrees with WORLD_SIZE={env_world}", file=sys.stderr)
        sys.exit(2)

    world = int(env_world or "1")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    local = local % torch.cuda.device_count() if args.backend == "gloo" else local
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)  # RCCL over xGMI
        else:
            dist.init_process_group("gloo")

    from vad_amd.ffn import TOPOLOGY_BL13, TOPOLOGY_REF39, FFNClassifier, random_layers
    from vad_amd.pipeline import VadPipeline
    from vad_amd.dist import LabelGather, any_rank

    topo = TOPOLOGY_BL13 if args.ffn == "bl13" else TOPOLOGY_REF39
    layers = random_layers(topo, seed=3)
    pipe = VadPipeline(FFNClassifier(layers))
    F = args.frames
    n_samples = 160 * (F - 1) + 401
    audio = synth_audio(n_samples, 100 + rank, dev)
    assert pipe.n_frames(audio.numel()) == F
    mfcc = torch.empty((F, 13), dtype=torch.float32, device=dev)
    labels = torch.empty((F - 5,), dtype=torch.uint8, device=dev)
    ffn_plan = pipe.ffn.plan
    stream = torch.cuda.current_stream()

    # N > 1: each step's decisions are gathered to rank 0 (RCCL over xGMI).
    # With nccl the gather of step k runs on RCCL's stream while step k + 1
    # computes: two label buffers, each reused only after its previous
    # gather completed (a stream-side wait, no host sync); every gather is
    # complete before the timed region ends.  gloo (the rehearsal on one GPU)
    # stages through the host and gathers synchronously.
    n_buf = max(args.streams, 2 if world > 1 else 1)
    labs = [labels] + [torch.empty_like(labels) for _ in range(n_buf - 1)]
    gathers = [LabelGather(F - 5, dev) for _ in labs] if world > 1 else []
    pend = [None] * len(labs)
    k_step = [0]
    # step k runs on streams[k % S] into label buffer k % n_buf; a buffer is
    # always written from the same stream (n_buf is a multiple of S or S = 1)
    streams = [stream] + [torch.cuda.Stream(device=dev) for _ in range(args.streams - 1)]
    for s in streams[1:]:
        s.wait_stream(stream)  # synth_audio wrote the clip on the default stream

    def step():
        # vad_mfcc_ffn with a workspace: the MFCC kernel, then the window
        # features + split-f16 MFMA FFN kernel (the faster of the two clip
        # forms on gfx950; the fused single kernel is timed below)
        i = k_step[0] % len(labs)
        k_step[0] += 1
        with torch.cuda.stream(streams[i % len(streams)]):
            if pend[i] is not None:
                pend[i].wait()
                pend[i] = None
            pipe.labels(audio, out=labs[i])
            if world > 1:
                pend[i] = gathers[i].start(labs[i], async_op=args.backend == "nccl")

    def drain():
        for i, w in enumerate(pend):
            if w is not None:
                w.wait()
                pend[i] = None

    t_w = time.perf_counter()
    for _ in range(args.warmup):
        step()
    drain()
    torch.cuda.synchronize()
    extra = 0
    # every step issues a gather (N > 1), a collective: all ranks must run
    # the same number of warm-up steps, so the time-based continuation is
    # agreed on before each batch (any rank still short of the minimum warm-up
    # keeps every rank going) -- a rank-local decision would leave the ranks'
    # collectives mismatched
    flag_dev = dev if args.backend == "nccl" else torch.device("cpu")
    while any_rank(time.perf_counter() - t_w < args.min_warmup_s, flag_dev):
        for _ in range(10):
            step()
        extra += 10
        drain()
        torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        step()
    drain()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=flag_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    # the same K steps strictly serial on one stream (no gathers): the latency
    # of one clip through both kernels, beside the pipelined headline
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ts = time.perf_counter()
    for k in range(args.steps):
        pipe.labels(audio, out=labels)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    ts = time.perf_counter() - ts
    if world > 1:
        t = torch.tensor([ts], dtype=torch.float64, device=flag_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ts = float(t.item())
    # per-kernel launch durations, right after the timed region: HIP events
    # around `steps` back-to-back launches of one kernel (an event record
    # between two kernels idles the GPU for ~5 us, so the timed steps carry
    # none)
    # (batches of 10 launches between event pairs: the mean over all of them,
    # and p10 / p50 / p90 of the batch means; at least 30 batches, so that one
    # slow batch -- a clock dip, a neighbour's burst on the node -- moves the
    # mean by a thirtieth of its excess rather than a tenth)
    def kernel_ms(fn, batch=10):
        nb = max(30, args.steps // batch)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(nb + 1)]
        ev[0].record(stream)
        for i in range(nb):
            for _ in range(batch):
                fn()
            ev[i + 1].record(stream)
        torch.cuda.synchronize()
        per = sorted(ev[i].elapsed_time(ev[i + 1]) / batch for i in range(nb))
        pct = {f"p{q}": per[min(nb - 1, int(q / 100 * nb))] for q in (10, 50, 90)}
        return ev[0].elapsed_time(ev[nb]) / (nb * batch), pct
    # N > 1: the gather alone ("plus gather time"), every rank
    # issuing `steps` back-to-back gathers of its F - 5 uint8 labels to rank 0,
    # synchronised and max-reduced like the timed region; the timed steps
    # above overlap each gather with the next step's kernels
    gather = None
    if world > 1:
        n_g = max(10, args.steps)
        dist.barrier()
        torch.cuda.synchronize()
        tg = time.perf_counter()
        for _ in range(n_g):
            gathers[0].start(labs[0], async_op=False)
        torch.cuda.synchronize()
        dist.barrier()
        tg = time.perf_counter() - tg
        t = torch.tensor([tg], dtype=torch.float64, device=flag_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        gather = {"gather_ms": float(t.item()) * 1e3 / n_g, "label_bytes_per_rank": F - 5,
                  "collective": "gather" if gathers[0].use_gather else "all_gather",
                  "backend": args.backend, "gathers_timed": n_g,
                  "note": "standalone (host-timed, max over ranks); in the timed steps each gather "
                          + ("overlaps the next step's kernels on RCCL's stream" if args.backend == "nccl"
                             else "runs through gloo's host path (rehearsal backend)")}
    mfcc_ms, mfcc_pct = kernel_ms(lambda: pipe.mfcc(audio, out=mfcc))
    ffn_ms, ffn_pct = kernel_ms(lambda: ffn_plan.window_labels(mfcc, out=labels))
    # the fused single-kernel clip form (MFCC rows kept on chip) and the FFN
    # on exact-f32 MFMA, beside the headline's forms
    fused_ms, fused_pct = kernel_ms(lambda: pipe.labels(audio, out=labels, fused=True))
    exact = FFNClassifier(layers, arith="f32")
    ffn_f32_ms, _ = kernel_ms(lambda: exact.plan.window_labels(mfcc, out=labels))
    del exact
    # the same clip as int16 PCM (what vad.py reads; exact: the samples are
    # integers in the int16 range), MFCC kernel only -- reported beside `value`
    audio16 = audio.to(torch.int16)
    mfcc16 = torch.empty_like(mfcc)
    for _ in range(10):
        pipe.mfcc(audio16, out=mfcc16)
    mfcc16_ms, _ = kernel_ms(lambda: pipe.mfcc(audio16, out=mfcc16))
    # the whole C3 step on that int16 clip (bit-identical labels, tested),
    # pipelined over the same streams and label buffers as the headline;
    # reported beside `value`, which stays the fp32-input step
    def step16(k):
        with torch.cuda.stream(streams[k % len(streams)]):
            pipe.labels(audio16, out=labs[k % len(labs)])
    for k in range(20):
        step16(k)
    torch.cuda.synchronize()
    t16 = time.perf_counter()
    for k in range(args.steps):
        step16(k)
    torch.cuda.synchronize()
    step16_ms = (time.perf_counter() - t16) * 1e3 / args.steps
    del audio16

    if rank == 0:
        value = world * F * args.steps / el
        dom_ms, dom_bytes, dom = (mfcc_ms, MFCC_BYTES_PER_FRAME, "mfcc_kernel") \
            if mfcc_ms >= ffn_ms else (ffn_ms, FFN_BYTES_PER_FRAME, "ffn_kernel")
        achieved = dom_bytes * F / (dom_ms * 1e-3) / 1e9
        # roofline.traffic is NOT measured in this run (a PMC pass cannot run
        # inside the timed process): it is read from the committed rocprofv3
        # --pmc FETCH_SIZE / WRITE_SIZE pass (profiles/pmc_traffic.json), and
        # traffic_source says which run produced it
        traffic, traffic_source = None, None
        tp = os.path.join(REPO, "profiles", "pmc_traffic.json")
        if os.path.exists(tp):
            with open(tp) as f:
                tj = json.load(f)
            traffic = tj.get(dom, {}).get("hbm_bytes_per_launch")
            if traffic is not None:
                traffic_source = {"file": "profiles/pmc_traffic.json", "measured_in_this_run": False,
                                  "run": tj.get("source"), "kernel": tj.get(dom, {}).get("kernel"),
                                  "correction": tj.get("correction")}
        out = {
            "metric": "MFCC+FFN frames/sec on 16 kHz 25 ms/10 ms hop",
            "value": value,
            "unit": "frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "warmup_extra_steps": extra,
            "ms_per_step": el * 1e3 / args.steps,
            "ms_per_step_note": (f"pipelined throughput: consecutive steps alternate over {args.streams} HIP "
                                 "streams, so a step's MFCC overlaps the previous step's FFN; "
                                 "ms_per_step_serial is the same K steps on one stream")
            if args.streams > 1 else "steps serial on one stream",
            "ms_per_step_serial": ts * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "dtype_detail": "MFCC: fp32 (packed-fp32 VALU FFT, fp32 mel / log10 / DCT); FFN: split-f16x3 "
                            "MFMA (v_mfma_f32_16x16x32_f16 on hi/lo f16 halves of every operand, "
                            "lo*hi + hi*lo + hi*hi, f32 accumulate; logit error within 1.5x of an "
                            "exact-f32 forward, tests/test_gpu_fullsize.py); exact-f32 FFN timed in "
                            "kernels_ms.ffn_kernel_exact_f32",
            "data": "synthetic (int16-range noise, 10**U(0,4) segment gains, 5% digital silence; "
                    "seeded random-init FFN weights)",
            "config": {"workload": "C3/C4: MFCC + FFN VAD forward, 1 clip of F frames per GPU "
                                   "(25 ms frames, 10 ms hop, 512-pt FFT, 26 mel, 13 MFCC, "
                                   "analyser 5-frame features), labels gathered to rank 0",
                       "frames_per_gpu": F, "ffn": "-".join(map(str, topo)),
                       "hip_streams": args.streams,
                       "parallelism": f"clip-shard x{world}"},
            "roofline": {"bound": "hbm", "kernel": dom,
                         "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "traffic_source": traffic_source,
                         "frac_vs_measured_copy": achieved / HBM_COPY_GBS,
                         "algorithmic_bytes_per_launch": dom_bytes * F,
                         "avg_launch_ms": dom_ms},
            # the MFCC kernel sits at the fp32 ridge (~20 flop/B): its VALU
            # ceiling beside the HBM one
            "compute": {"bound": "valu", "kernel": "mfcc_kernel",
                        "achieved": MFCC_FLOPS_PER_FRAME * F / (mfcc_ms * 1e-3) / 1e12,
                        "peak": VALU_PEAK_TFS, "unit": "TFLOP/s",
                        "frac": MFCC_FLOPS_PER_FRAME * F / (mfcc_ms * 1e-3) / 1e12 / VALU_PEAK_TFS,
                        "flops_per_frame": MFCC_FLOPS_PER_FRAME},
            # the VALU time those instructions take at the measured rates,
            # against the kernel's measured launch time
            "valu_model": {"kernel": "mfcc_kernel",
                           "packed_per_frame": MFCC_VALU_PACKED_PER_FRAME,
                           "scalar_per_frame": MFCC_VALU_SCALAR_PER_FRAME,
                           "ns_packed": VALU_NS_PACKED_2W, "ns_scalar": VALU_NS_SCALAR_2W,
                           "model_ms": F / N_SIMDS * (MFCC_VALU_PACKED_PER_FRAME * VALU_NS_PACKED_2W
                                                      + MFCC_VALU_SCALAR_PER_FRAME * VALU_NS_SCALAR_2W) * 1e-6,
                           "frac_of_launch": F / N_SIMDS * (MFCC_VALU_PACKED_PER_FRAME * VALU_NS_PACKED_2W
                                                            + MFCC_VALU_SCALAR_PER_FRAME * VALU_NS_SCALAR_2W)
                           * 1e-6 / mfcc_ms},
            "kernels_ms": {"mfcc_kernel": mfcc_ms, "ffn_kernel": ffn_ms,
                           "ffn_kernel_exact_f32": ffn_f32_ms, "mfcc_ffn_fused_kernel": fused_ms},
            "kernels_ms_pct": {"mfcc_kernel": mfcc_pct, "ffn_kernel": ffn_pct,
                               "mfcc_ffn_fused_kernel": fused_pct},
            "mfcc_int16_input": {"avg_launch_ms": mfcc16_ms,
                                 "frames_per_s": F / (mfcc16_ms * 1e-3),
                                 "c3_step_ms": step16_ms,
                                 "c3_step_frames_per_s": world * F / (step16_ms * 1e-3) if world == 1 else None,
                                 "note": "int16 PCM (vad.py's wav samples before astype(float32)): the same "
                                         "clip, exact conversion, bit-identical MFCCs and labels",
                                 "algorithmic_bytes_per_frame": 160 * 2 + 13 * 4,
                                 "achieved_GBps": (160 * 2 + 13 * 4) * F / (mfcc16_ms * 1e-3) / 1e9},
        }
        if gather is not None:
            out["gather"] = gather
        if world == 1:
            out["feed_frame_latency"] = feed_frame_latency(dev)
            if not args.no_secondary:
                out["secondary_configs"] = secondary_configs(dev)
        if world == 1 and not args.no_cpu:
            out["cpu_baseline"] = cpu_baseline(layers)
            out["cpu_baseline_all_cores"] = cpu_baseline_all(tuple(topo))
            pf1, pfall = cpu_baseline_per_frame(tuple(topo))
            out["cpu_baseline_per_frame"] = pf1
            out["cpu_baseline_per_frame_all_cores"] = pfall
            out["cpu_host"] = host_facts()
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
