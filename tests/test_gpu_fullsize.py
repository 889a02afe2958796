"""The HIP path against the oracle at the benchmark configurations' full sizes
(SURVEY.md 8(d) configs C2, C3, C5), every frame and every window compared --
the multi-tile persistent loop of the MFCC kernel (a workgroup runs ~6 tiles
at 100k frames and ~61 at 1M), not only the single-tile case the fixtures hit.

Tolerances:
  MFCC    per frame ||d||_2/||ref||_2 <= 1e-4 and max|d| <= 1e-4 max|ref|
  labels  identical to the fp64 oracle wherever its top-2 logit margin
          exceeds LABEL_MARGIN; below it the disagreements are counted and
          bounded (a window's normalised features divide by its 5-frame std,
          so MFCC rounding ~1e-7 can move a near-tie)
  logits  split-f16 MFMA within SPLIT_VS_F32 x the error of the exact-f32
          MFMA forward, both against fp64 on the same device features
"""
import numpy as np
import pytest

from oracle import vad_oracle as O
from label_report import label_agreement, record_vs_baseline

pytestmark = pytest.mark.gpu

MFCC_TOL = 1e-4
LABEL_MARGIN = 0.05
SPLIT_VS_F32 = 2.5  # measured 1.05x (13-64-64-2) and 1.5x (39-64-32-16-3)
# the fp32-rounding margin: a window whose fp64 top-2 logit margin is below
# it may take either label (fp32 MFCC rounding ~1e-7 of a coefficient moves a
# normalised feature by up to ~1e-6 of the logit scale; round 4 measured its
# two disagreements at margins 3.2e-6 / 3.7e-6, profiles/r04/label_agreement_c3.json).
# Any legitimate change of fp32 summation order may flip a different subset
# of those near-ties, so the gate is the margin rule, not a frozen count:
# every disagreement sits below FP32_MARGIN, hence there are at most as many
# as there are windows below it.
FP32_MARGIN = 1e-5


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    return torch


def oracle_mfcc(clip, fb, chunk=100_000):
    """O.mfcc_batch over a long clip in frame chunks (same frames, bounded memory)."""
    F = O.n_frames(len(clip))
    out = []
    for f0 in range(0, F, chunk):
        f1 = min(F, f0 + chunk)
        out.append(O.mfcc_batch(clip[160 * f0: 160 * (f1 - 1) + 401], fb))
    return np.concatenate(out)


def assert_mfcc_close(got, ref):
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    assert got.shape == ref.shape
    d = got - ref
    rel = np.linalg.norm(d, axis=1) / np.linalg.norm(ref, axis=1)
    mx = np.abs(d).max(axis=1) / np.abs(ref).max(axis=1)
    assert rel.max() <= MFCC_TOL, (rel.max(), int(rel.argmax()))
    assert mx.max() <= MFCC_TOL, (mx.max(), int(mx.argmax()))
    return rel.max()


@pytest.mark.parametrize("nf", [26, 40])
def test_c2_mfcc_every_frame(torch_cuda, nf):
    """C2: 100k frames (1,563 tiles over the persistent workgroups), fp32 and
    int16 input, 26 and 40 filters, every frame vs the oracle."""
    torch = torch_cuda
    from vad_amd.plan import MfccPlan
    F = 100_000
    clip = O.synth_clip(O.samples_for_frames(F), seed=0)
    fb = O.get_mel_filterbanks(300, 8000, 512, nf, 16000)
    plan = MfccPlan(fb)
    assert plan.variant == (1 if nf == 26 else 2)
    a32 = torch.from_numpy(clip).cuda()
    m32 = plan.clip_mfcc(a32)
    m16 = plan.clip_mfcc(a32.to(torch.int16))
    assert torch.equal(m32, m16)  # the int16 load converts exactly
    ref = oracle_mfcc(clip, fb)
    assert_mfcc_close(m32.cpu().numpy(), ref)
    # the runtime-table kernel over the same frames
    plan.set_variant(0)
    assert_mfcc_close(plan.clip_mfcc(a32).cpu().numpy(), ref)


@pytest.mark.parametrize("word", ["0x80ff80ff80ff80ff", "0xffffffffffffff80", "0x8090a0b0c0d0e0ff"])
@pytest.mark.parametrize("F", [100_000, 12_345, 300])
def test_xcd_balanced_runs_cover_every_frame(torch_cuda, monkeypatch, word, F):
    """The MFCC kernel's XCD-balanced tile runs (vad_common.h MfccBalance)
    partition the tiles exactly whatever the weights: forced extreme weights
    give bit-identical MFCCs to equal runs, for grids of 256 workgroups and
    of fewer (12,345 frames: 193; 300: 5), and the adaptive default too."""
    torch = torch_cuda
    from vad_amd.plan import MfccPlan
    clip = O.synth_clip(O.samples_for_frames(F), seed=5)
    fb = O.get_mel_filterbanks(300, 8000, 512, 26, 16000)
    a32 = torch.from_numpy(clip).cuda()
    monkeypatch.setenv("VAD_MFCC_BALANCE", "0")
    want = MfccPlan(fb).clip_mfcc(a32)
    monkeypatch.setenv("VAD_MFCC_BALANCE", "1")
    adaptive = MfccPlan(fb)
    for _ in range(4):  # weights adapt from the stats of the launches before
        assert torch.equal(adaptive.clip_mfcc(a32), want)
    monkeypatch.setenv("VAD_MFCC_BALANCE_WORD", word)
    assert torch.equal(MfccPlan(fb).clip_mfcc(a32), want)


def test_c3_full_clip_vs_oracle(torch_cuda):
    """C3 (BASELINE configs[2]): 1M frames, 13-64-64-2 with the bench's
    weights; MFCCs of every frame and labels of every window vs the oracle
    (MFCC -> analyser features -> FFN, all fp64 after the f32 FFT), through
    both clip forms (two kernels / fused)."""
    torch = torch_cuda
    from vad_amd.ffn import TOPOLOGY_BL13, FFNClassifier, random_layers
    from vad_amd.pipeline import VadPipeline
    from vad_amd.plan import window_features
    F = 1_000_000
    clip = O.synth_clip(O.samples_for_frames(F), seed=1)
    layers = random_layers(TOPOLOGY_BL13, seed=3)
    pipe = VadPipeline(FFNClassifier(layers))
    a = torch.from_numpy(clip).cuda()
    m = pipe.mfcc(a)
    lab = pipe.labels(a)
    lab_fused = pipe.labels(a, fused=True)
    assert torch.equal(lab, lab_fused)
    fb = O.get_mel_filterbanks(300, 8000, 512, 26, 16000)
    ref_m = oracle_mfcc(clip, fb)
    assert_mfcc_close(m.cpu().numpy(), ref_m)
    got = lab.cpu().numpy()
    x = O.analyser_features_fast(ref_m)[:, :13]
    ref_l = O.ffn_labels(x, layers)
    marg = O.ffn_margin(x, layers)
    assert got.shape == ref_l.shape == (F - 5,)
    sure = marg > LABEL_MARGIN
    rep = label_agreement(got, ref_l, marg, name="label_agreement_c3",
                          extra={"config": "C3 1M frames, 13-64-64-2 seed 3, clip seed 1",
                                 "below_label_margin": int((~sure).sum()), "label_margin": LABEL_MARGIN})
    np.testing.assert_array_equal(got[sure], ref_l[sure])
    # the margin rule: every disagreement sits at the fp32-vs-fp64 MFCC
    # rounding scale, so their number is bounded by the near-tie windows
    assert all(d["margin"] < FP32_MARGIN for d in rep["disagree_windows"]), rep["disagree_windows"]
    n_near = int((marg < FP32_MARGIN).sum())
    assert rep["disagree"] <= n_near, (rep["disagree"], n_near)
    record_vs_baseline("c3_label_disagree", {"c3_label_disagree": rep["disagree"]})
    print(f"C3 labels: {rep['disagree']} of {F - 5} windows differ from the fp64 oracle, "
          f"{n_near} windows below the fp32 margin {FP32_MARGIN}")
    # and exactly the oracle's FFN on the device's own features where the
    # margin clears the forward's rounding
    xg = window_features(m).cpu().numpy()[:, :13]
    ok = O.ffn_margin(xg, layers) > 1e-4
    np.testing.assert_array_equal(got[ok], O.ffn_labels(xg, layers)[ok])
    assert ok.mean() > 0.999
    assert np.isnan(x).any(axis=1).sum() > 0  # digital silence exercised


@pytest.mark.parametrize("n_streams", [2, 3])
def test_c3_steps_alternating_streams(torch_cuda, n_streams):
    """bench.py's pipelined step: consecutive 1M-frame clips alternate over
    HIP streams (a workspace and a label buffer per stream, issued under
    torch.cuda.stream), so one clip's MFCC overlaps the previous clip's
    FFN; every buffer ends with the labels of the serial form, bit for bit."""
    torch = torch_cuda
    from vad_amd.ffn import TOPOLOGY_BL13, FFNClassifier, random_layers
    from vad_amd.pipeline import VadPipeline
    F = 1_000_000
    clips = [torch.from_numpy(O.synth_clip(O.samples_for_frames(F), seed=s)).cuda() for s in (1, 2)]
    pipe = VadPipeline(FFNClassifier(random_layers(TOPOLOGY_BL13, seed=3)))
    want = [pipe.labels(c).clone() for c in clips]
    streams = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(n_streams - 1)]
    labs = [torch.empty_like(want[0]) for _ in streams]
    for k in range(4 * n_streams + 1):  # clips alternate too: a buffer's last clip is k % 2
        with torch.cuda.stream(streams[k % n_streams]):
            pipe.labels(clips[k % 2], out=labs[k % n_streams])
    torch.cuda.synchronize()
    last = {k % n_streams: k % 2 for k in range(4 * n_streams + 1)}
    for i, lab in enumerate(labs):
        assert torch.equal(lab, want[last[i]]), i


@pytest.mark.parametrize("kernel", ["hop", "three"])
def test_c5_512_streams_graph_replay(torch_cuda, golden, kernel):
    """C5: 512 concurrent streams, 40 hops of 10 ms each as hipGraph replays
    (frame assembly + MFCC + features + FFN), every stream's labels vs the
    oracle's feed_frame semantics on that stream's audio."""
    torch = torch_cuda
    from vad_amd.ffn import FFNClassifier
    from vad_amd.stream import StreamBatch
    w = golden("ffn")
    layers = [(w[f"ref39_W{i}"], w[f"ref39_b{i}"]) for i in range(4)]
    S, T = 512, 40
    clips = np.stack([O.synth_clip(160 * (T - 1) + 401, seed=500 + s) for s in range(S)])
    sb = StreamBatch(S, FFNClassifier(layers), kernel=kernel)
    sb.prime(torch.from_numpy(np.ascontiguousarray(clips[:, :240])).cuda())
    sb.capture()
    # the one-hop capture is one kernel node, replayed as that node; the
    # three-kernel step goes through hipGraphLaunch
    assert sb.graph_direct == (kernel == "hop")
    hops = torch.from_numpy(np.ascontiguousarray(
        np.stack([clips[:, 240 + 160 * t: 400 + 160 * t] for t in range(T)]))).cuda()
    got = np.stack([sb.step(hops[t]).cpu().numpy().copy() for t in range(T)], axis=1)  # (S, T)
    assert (got[:, :5] == 255).all()
    fb = O.get_mel_filterbanks(300, 8000, 512, 26, 16000)
    ref_l, marg = [], []
    for s in range(S):
        x = O.analyser_features_fast(O.mfcc_batch(clips[s], fb))
        ref_l.append(O.ffn_labels(x, layers))
        marg.append(O.ffn_margin(x, layers))
    ref_l, marg = np.stack(ref_l), np.stack(marg)  # (S, T-5)
    # the MFCC ring the streams hold equals the oracle's last five frames
    ring = sb.ring.cpu().numpy()
    cnt = sb.count.cpu().numpy()
    for s in range(0, S, 37):
        want = O.mfcc_batch(clips[s], fb)[-5:]
        got_rows = np.stack([ring[s][(cnt[s] + d) % 5] for d in range(5)])
        rel = np.linalg.norm(got_rows - want, axis=1) / np.linalg.norm(want, axis=1)
        assert rel.max() <= MFCC_TOL, (s, rel.max())
    sure = marg > LABEL_MARGIN
    np.testing.assert_array_equal(got[:, 5:][sure], ref_l[sure])
    assert int((got[:, 5:] != ref_l).sum()) <= 2


def test_stream_hops_100k_streams(torch_cuda, golden):
    """Maximum-size edge of the streaming path: 100,000 live streams (16
    streams per block, 6,250 blocks), 8 hops as one vad_stream_hops launch
    and as 8 one-hop launches on a second batch: identical labels, frames,
    rings and counts; every 997th stream's labels vs the oracle's (margin
    rule) and its frame buffer equal to the last 400 samples it was fed."""
    torch = torch_cuda
    from vad_amd.ffn import FFNClassifier
    from vad_amd.stream import StreamBatch
    w = golden("ffn")
    layers = [(w[f"ref39_W{i}"], w[f"ref39_b{i}"]) for i in range(4)]
    S, T = 100_000, 8
    n = 160 * (T - 1) + 401
    g = torch.Generator(device="cuda").manual_seed(79)
    amp = 10.0 ** (4 * torch.rand((S, 1), generator=g, device="cuda"))
    clips = (torch.randn((S, n), generator=g, device="cuda") * amp).round_().clamp_(-32767, 32767)
    hops = clips[:, 240:240 + 160 * T].reshape(S, T, 160).transpose(0, 1).contiguous()  # (T, S, 160)
    clf = FFNClassifier(layers)
    blk = StreamBatch(S, clf, kernel="hop", hops_per_step=T)
    one = StreamBatch(S, clf, kernel="hop")
    for sb in (blk, one):
        sb.prime(clips[:, :240].contiguous())
    lab_blk = blk.step_block(hops).clone()  # (T, S)
    lab_one = torch.stack([one.step(hops[t]).clone() for t in range(T)])
    assert torch.equal(lab_blk, lab_one)
    for a, b in ((blk.frames, one.frames), (blk.ring, one.ring), (blk.count, one.count)):
        assert torch.equal(a, b)
    assert torch.equal(blk.frames, clips[:, n - 401: n - 1])  # the last frame fed: samples 160 (T-1) ..
    assert (lab_blk[:5] == 255).all()
    fb = O.get_mel_filterbanks(300, 8000, 512, 26, 16000)
    got = lab_blk[5:].cpu().numpy()  # (T - 5, S)
    n_ok = 0
    for s in range(0, S, 997):
        c = clips[s].cpu().numpy()  # T frames (strict '>' framing): windows 0 .. T - 6
        x = O.analyser_features_fast(O.mfcc_batch(c, fb))
        ok = O.ffn_margin(x, layers) > LABEL_MARGIN
        np.testing.assert_array_equal(got[:, s][ok], O.ffn_labels(x, layers)[ok])
        n_ok += int(ok.sum())
    assert n_ok > 0.9 * 3 * len(range(0, S, 997))
    del clips, hops, blk, one
    torch.cuda.empty_cache()


@pytest.mark.parametrize("topo", [(13, 64, 64, 2), (39, 64, 32, 16, 3)])
def test_split_f16_logit_error_bounded(torch_cuda, topo):
    """The split-f16 MFMA forward (hi*hi + hi*lo + lo*hi, lo*lo dropped)
    against fp64 on the device's own features: its worst logit error is
    within SPLIT_VS_F32 x that of the exact-f32 MFMA forward (and both are
    f32-rounding sized)."""
    torch = torch_cuda
    from vad_amd.ffn import FFNClassifier, random_layers
    from vad_amd.pipeline import VadPipeline
    from vad_amd.plan import window_features, window_logits
    F = 50_000
    clip = O.synth_clip(O.samples_for_frames(F), seed=31)
    layers = random_layers(topo, seed=5)
    m = VadPipeline().mfcc(torch.from_numpy(clip).cuda())
    x = window_features(m).cpu().numpy()[:, :topo[0]]
    z64, _ = O.ffn_forward(x, layers)
    fin = np.isfinite(z64).all(axis=1)
    scale = np.abs(z64[fin]).max()
    err = {}
    for arith in ("split_f16", "f32"):
        clf = FFNClassifier(layers, arith=arith)
        assert clf.arith == arith
        labels, logits = window_logits(clf.plan, m)
        z = logits.cpu().numpy().astype(np.float64)
        assert np.array_equal(np.isnan(z).any(axis=1), ~fin)  # NaN windows stay NaN
        err[arith] = np.abs(z[fin] - z64[fin]).max() / scale
        np.testing.assert_array_equal(labels.cpu().numpy(), O.ffn_labels(z.astype(np.float32), [(np.eye(z.shape[1]), np.zeros(z.shape[1]))]))
    print(f"logit error / max|logit|: split-f16 {err['split_f16']:.3e}, exact f32 {err['f32']:.3e}")
    assert err["f32"] < 1e-5
    assert err["split_f16"] <= SPLIT_VS_F32 * err["f32"], err


def test_clip_past_2g_samples(torch_cuda):
    """Maximum-size edge: a 14M-frame clip (2.24e9 samples, 9 GB of fp32 and
    4.5 GB of int16 on the device) takes sample offsets past 2^31 and byte
    offsets past 2^32.  Every frame's computation is position independent,
    so windows of the big clip, at its start, across sample 2^31 and at its
    end, equal (bit for bit) the same frames cut out as small clips: MFCCs
    (fp32 and int16 input) and the two-kernel labels.  Size-independent
    property check: the oracle stays at the small sizes of the other tests."""
    torch = torch_cuda
    from vad_amd.ffn import TOPOLOGY_BL13, FFNClassifier, random_layers
    from vad_amd.pipeline import VadPipeline
    free, _ = torch.cuda.mem_get_info()
    if free < 24 << 30:
        pytest.skip("needs ~24 GB of free device memory")
    F = 14_000_000
    n = 160 * (F - 1) + 401
    assert n > 2 ** 31
    g = torch.Generator(device="cuda").manual_seed(77)
    audio = (torch.randn(n, generator=g, device="cuda") * 3000).round_().clamp_(-32767, 32767)
    pipe = VadPipeline(FFNClassifier(random_layers(TOPOLOGY_BL13, seed=3)))
    big = pipe.mfcc(audio)
    big_lab = pipe.labels(audio)
    a16 = audio.to(torch.int16)
    assert torch.equal(pipe.mfcc(a16), big)
    del a16
    W = 2000  # frames per cut
    for f0 in (0, (2 ** 31) // 160 - W // 2, F - W):
        cut = audio[160 * f0: 160 * (f0 + W - 1) + 401].contiguous()
        assert torch.equal(pipe.mfcc(cut), big[f0:f0 + W]), f0
        assert torch.equal(pipe.labels(cut), big_lab[f0:f0 + W - 5]), f0
    del audio, big, big_lab
    torch.cuda.empty_cache()


def test_clip_past_2g_mfcc_values(torch_cuda):
    """Maximum-size edge, one step further: 170M frames of int16 PCM (27.2e9
    samples, 54 GB on the device; 8.8 GB of MFCC rows) put the MFCC row
    element index 13 f past 2^31 (at frame 165,191,050) and the window
    index of the FFN and fused kernels past 2^27 tiles.  As above, frames cut
    out of the big clip at its start, across that boundary and at its end
    give bit-identical MFCCs and labels as small clips; the fused kernel's
    labels equal the two-kernel labels over the whole clip."""
    torch = torch_cuda
    from vad_amd.ffn import TOPOLOGY_BL13, FFNClassifier, random_layers
    from vad_amd.pipeline import VadPipeline
    free, _ = torch.cuda.mem_get_info()
    if free < 100 << 30:
        pytest.skip("needs ~100 GB of free device memory")
    F = 170_000_000
    n = 160 * (F - 1) + 401
    assert 13 * F > 2 ** 31
    g = torch.Generator(device="cuda").manual_seed(78)
    a16 = torch.randint(-32767, 32768, (n,), dtype=torch.int16, device="cuda", generator=g)
    a16[160 * (F - 3000): 160 * (F - 2000)] = 0  # digital silence near the end: NaN windows
    pipe = VadPipeline(FFNClassifier(random_layers(TOPOLOGY_BL13, seed=3)))
    assert pipe.fusable
    big = pipe.mfcc(a16)
    big_lab = pipe.labels(a16)
    assert torch.equal(pipe.labels(a16, fused=True), big_lab)
    W = 4000  # frames per cut
    for f0 in (0, (2 ** 31) // 13 - W // 2, F - W):
        cut = a16[160 * f0: 160 * (f0 + W - 1) + 401].contiguous()
        assert torch.equal(pipe.mfcc(cut), big[f0:f0 + W]), f0
        assert torch.equal(pipe.labels(cut), big_lab[f0:f0 + W - 5]), f0
    assert (big_lab[F - 2990: F - 2010] == 0).all()  # windows inside the silence
    del a16, big, big_lab
    torch.cuda.empty_cache()


def test_kernel_time_guard(torch_cuda):
    """A coarse regression guard on the benchmark kernels (C3 sizes, 1M
    frames), reported rather than tuned: the median over 7 batches of 20
    launches (after a 0.3 s warm-up) must stay under 2x the round-4 driver's
    times (MFCC 0.245 ms, FFN 0.052 ms), so only a gross regression (a
    spill, a lost specialisation) fails the correctness run; XCD clock dips
    and neighbour bursts move single batches by ~15 %, which the median and
    the 2x bound absorb.  The bench, not this test, measures performance."""
    import time
    torch = torch_cuda
    from vad_amd.ffn import TOPOLOGY_BL13, FFNClassifier, random_layers
    from vad_amd.pipeline import VadPipeline
    F = 1_000_000
    clip = O.synth_clip(O.samples_for_frames(F), seed=1)
    pipe = VadPipeline(FFNClassifier(random_layers(TOPOLOGY_BL13, seed=3)))
    a = torch.from_numpy(clip).cuda()
    m = torch.empty((F, 13), dtype=torch.float32, device="cuda")
    lab = torch.empty((F - 5,), dtype=torch.uint8, device="cuda")
    plan = pipe.ffn.plan

    def median_ms(fn, batches=7, reps=20):
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 0.3:
            fn()
            torch.cuda.synchronize()
        out = []
        for _ in range(batches):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(reps):
                fn()
            e.record()
            torch.cuda.synchronize()
            out.append(s.elapsed_time(e) / reps)
        return float(np.median(out))

    t_mfcc = median_ms(lambda: pipe.mfcc(a, out=m))
    t_ffn = median_ms(lambda: plan.window_labels(m, out=lab))
    print(f"kernel time guard: MFCC {t_mfcc * 1e3:.1f} us, FFN {t_ffn * 1e3:.1f} us per 1M frames")
    # recorded beside the previous round's driver times, increases flagged
    # (gpurun_out/kernel_time_guard.json)
    record_vs_baseline("kernel_time_guard", {"mfcc_kernel_ms": t_mfcc, "ffn_kernel_ms": t_ffn})
    assert t_mfcc < 2 * 0.245, t_mfcc
    assert t_ffn < 2 * 0.052, t_ffn
