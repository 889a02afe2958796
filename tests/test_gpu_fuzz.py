"""Property-based (hypothesis) fuzzing of the HIP clip and streaming paths
against the oracle (test plan item 2: "HIP vs the CPU
restatement, with hypothesis-fuzzed clip lengths and amplitudes").

Each example draws a clip length (0 .. 30k samples, so frame counts around
the 64-frame tiles, the framing edges L = 400 / 401 / 560 / 561 and clips too
short for a window), an amplitude 10^U(-2, 4.6) (clipped to the int16 range),
an optional digital-silence span (NaN windows), float32 or int16 input,
the analyser or offline feature form and a fixture network, then checks:

  frame count      O.n_frames (split_into_frames' strict '>', A3)
  MFCC             the oracle's per-frame rule (MFCC_TOL, test_gpu_parity)
  int16 input      bit-identical MFCCs and labels to the same samples as fp32
  features         NaN positions and values of the oracle's features of the
                   device MFCCs (offline: 1e-5 of the row norm; analyser: the
                   NaN pattern, the values being test_gpu_features_parity's)
  labels           the oracle's forward on the device features wherever its
                   top-2 margin exceeds MARGIN_TOL; the fused kernel's labels
                   identical to the two-kernel form's
  streaming        a StreamBatch fed the same clips hop by hop (random stream
                   count and hops per call) gives the clip path's labels
                   wherever the margin is decisive

derandomize=True: every run draws the same examples (no flaky GPU runs);
database=None: nothing is written next to the tests.  A deep run
(VAD_FUZZ_SCALE=k, VAD_FUZZ_SEED=s) draws k times the examples from seed s
instead -- a search for new defects, not part of the round-end suite.
"""
import os
import numpy as np
import pytest

from oracle import vad_oracle as O

hyp = pytest.importorskip("hypothesis")
from hypothesis import HealthCheck, given, settings  # noqa: E402
from hypothesis import strategies as st  # noqa: E402

pytestmark = pytest.mark.gpu

MFCC_TOL = 1e-4
MARGIN_TOL = 0.05
_SCALE = int(os.environ.get("VAD_FUZZ_SCALE", "1"))
_SEED = os.environ.get("VAD_FUZZ_SEED")
FUZZ = settings(max_examples=120 * _SCALE, deadline=None, derandomize=_SEED is None, database=None,
                suppress_health_check=[HealthCheck.function_scoped_fixture, HealthCheck.too_slow])


def fuzz(n):
    """The suite's settings with n examples per test (times VAD_FUZZ_SCALE);
    with VAD_FUZZ_SEED the examples come from that seed."""
    s = settings(FUZZ, max_examples=n * _SCALE)
    return s if _SEED is None else (lambda f: hyp.seed(int(_SEED))(s(f)))


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    return torch


@pytest.fixture(scope="module")
def nets(golden):
    w = golden("ffn")
    return {p: [(w[f"{p}_W{i}"], w[f"{p}_b{i}"]) for i in range(n)] for p, n in (("ref39", 4), ("bl13", 3))}


def fuzz_clip(n, log_amp, seed, silence, integral):
    rng = np.random.default_rng(seed)
    x = rng.standard_normal(n) * 10.0 ** log_amp
    if silence is not None and n > 0:
        a, b = sorted(int(f * n) for f in silence)
        x[a:b] = 0.0
    x = np.clip(x, -32767.0, 32767.0)
    if integral:
        x = np.rint(x)
    return x.astype(np.float32)


def mel_conditioned(frames, fft_n, fb):
    """Frames whose every mel energy stands clear of the FFT's rounding noise:
    min_m e_m >= 1e-9 max_m e_m over the bank's non-empty filters (or the
    frame is silent).  A band on an exact spectral null -- a frame of two
    +-1 samples d apart zeroes every bin k with k d / fft_n integral -- has
    energy 0 in exact arithmetic and float32 rounding noise in the oracle's
    (the reference's) FFT: 1.4e-37 where the device's DFT gives 0 -> eps, so
    that filter's log-energy, and the MFCC, are the noise's, not the
    signal's.  Found by a deep fuzz run (VAD_FUZZ_SEED=9001: frame_len 115,
    stride 92, fft_n 300, 40 filters, amplitude 10^-0.75 rounded to
    integers); the tolerance of the other frames is unchanged."""
    frames = list(frames)
    if not frames:
        return np.zeros(0, bool)
    spec = O.spec_batch(np.stack(frames), fft_n).astype(np.float64)
    e = spec @ fb[fb.sum(axis=1) > 0].T
    emax = e.max(axis=1)
    return (emax == 0) | (e.min(axis=1) >= 1e-9 * emax)


def assert_mfcc_close(got, ref, floor=None):
    """The MFCC tolerance (test_gpu_parity): per frame ||d|| <= 1e-4 ||ref||
    and max |d| <= 1e-4 max |ref|.  floor (per frame) bounds both
    denominators from below -- for banks where the kept coefficients can
    cancel (test_fuzz_get_mfcc_any_bank)."""
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    assert got.shape == ref.shape
    if len(ref) == 0:
        return
    d = got - ref
    fl = 0.0 if floor is None else np.asarray(floor, np.float64)
    rel = np.linalg.norm(d, axis=1) / np.maximum(np.linalg.norm(ref, axis=1), fl)
    mx = np.abs(d).max(axis=1) / np.maximum(np.abs(ref).max(axis=1), fl)
    assert rel.max() <= MFCC_TOL, (rel.max(), int(rel.argmax()))
    assert mx.max() <= MFCC_TOL, (mx.max(), int(mx.argmax()))


@fuzz(120)
@given(n=st.one_of(st.integers(0, 30000), st.sampled_from([0, 399, 400, 401, 560, 561, 1200, 1201, 10481])),
       log_amp=st.floats(-2.0, 4.6), seed=st.integers(0, 2 ** 32 - 1),
       silence=st.one_of(st.none(), st.tuples(st.floats(0, 1), st.floats(0, 1))),
       i16=st.booleans(), offline=st.booleans(), topo=st.sampled_from(["ref39", "bl13"]))
def test_fuzz_clip_path(torch_cuda, nets, n, log_amp, seed, silence, i16, offline, topo):
    import torch
    from vad_amd import _lib
    from vad_amd import plan as P
    from vad_amd.ffn import FFNClassifier
    from vad_amd.pipeline import VadPipeline
    clip = fuzz_clip(n, log_amp, seed, silence, integral=i16)
    lay = nets[topo]
    pipe = VadPipeline(FFNClassifier(lay), mode="offline" if offline else "analyser")
    a = torch.from_numpy(np.resize(clip, max(n, 1))).cuda()[:n]  # n = 0: a valid empty tensor
    F = O.n_frames(n)
    m = pipe.mfcc(a)
    assert m.shape == (F, 13)
    mc = m.cpu().numpy()
    fb = O.get_mel_filterbanks(300, 8000, 512, 26, 16000)
    ok = mel_conditioned(O.frame_matrix(clip), 512, fb)
    assert_mfcc_close(mc[ok], (O.mfcc_batch(clip, fb) if F else np.zeros((0, 13)))[ok])
    lab = pipe.labels(a).cpu().numpy()
    assert lab.shape == (max(F - 5, 0),)
    if i16:
        a16 = torch.from_numpy(np.resize(clip.astype(np.int16), max(n, 1))).cuda()[:n]
        assert torch.equal(pipe.mfcc(a16), m)
        np.testing.assert_array_equal(pipe.labels(a16).cpu().numpy(), lab)
    if pipe.fusable:
        np.testing.assert_array_equal(pipe.labels(a, fused=True).cpu().numpy(), lab)
    if F <= 5:
        return
    mode = _lib.FEAT_OFFLINE if offline else _lib.FEAT_ANALYSER
    x = P.window_features(m, mode).cpu().numpy().astype(np.float64)
    if offline:
        ref = O.offline_features(mc).reshape(F - 5, 39)
        err = np.linalg.norm(x - ref, axis=1) / np.maximum(np.linalg.norm(ref, axis=1), 1e-30)
        assert err.max() <= 1e-5
    else:
        ref = O.analyser_features_fast(mc)
        np.testing.assert_array_equal(np.isnan(x), np.isnan(ref))
    x = x[:, :lay[0][0].shape[0]]
    ok = O.ffn_margin(x, lay) > MARGIN_TOL
    np.testing.assert_array_equal(lab[ok], O.ffn_labels(x, lay)[ok])


@fuzz(12)
@given(F=st.integers(2_000, 120_000), tail=st.integers(0, 159), log_amp=st.floats(-1.0, 4.6),
       seed=st.integers(0, 2 ** 32 - 1), silence=st.one_of(st.none(), st.tuples(st.floats(0, 1), st.floats(0, 1))),
       offline=st.booleans(), topo=st.sampled_from(["ref39", "bl13"]))
def test_fuzz_large_clip_partitions(torch_cuda, nets, F, tail, log_amp, seed, silence, offline, topo):
    """Clips of 2k..120k frames: the MFCC kernel's runs of 64-frame tiles and
    the fused kernel's window ranges [n_win b / G, n_win (b + 1) / G) fall at
    arbitrary places (test_fuzz_clip_path's clips give most workgroups one
    tile or none, the full-size tests a few fixed sizes).  Every frame's MFCC
    vs the oracle, fused labels == two-kernel labels, int16 == fp32, labels
    vs the oracle's forward where its margin is decisive."""
    import torch
    from vad_amd import _lib
    from vad_amd import plan as P
    from vad_amd.ffn import FFNClassifier
    from vad_amd.pipeline import VadPipeline
    n = 160 * (F - 1) + 401 + tail
    clip = fuzz_clip(n, log_amp, seed, silence, integral=True)
    assert O.n_frames(n) == F
    lay = nets[topo]
    pipe = VadPipeline(FFNClassifier(lay), mode="offline" if offline else "analyser")
    a = torch.from_numpy(clip).cuda()
    m = pipe.mfcc(a)
    mc = m.cpu().numpy()
    fb = O.get_mel_filterbanks(300, 8000, 512, 26, 16000)
    ok = mel_conditioned(O.frame_matrix(clip), 512, fb)
    assert_mfcc_close(mc[ok], O.mfcc_batch(clip, fb)[ok])
    lab = pipe.labels(a).cpu().numpy()
    assert torch.equal(pipe.mfcc(a.to(torch.int16)), m)
    if pipe.fusable:
        np.testing.assert_array_equal(pipe.labels(a, fused=True).cpu().numpy(), lab)
    mode = _lib.FEAT_OFFLINE if offline else _lib.FEAT_ANALYSER
    x = P.window_features(m, mode).cpu().numpy().astype(np.float64)[:, :lay[0][0].shape[0]]
    okl = O.ffn_margin(x, lay) > MARGIN_TOL
    np.testing.assert_array_equal(lab[okl], O.ffn_labels(x, lay)[okl])
    assert okl.mean() > 0.5


@fuzz(50)
@given(S=st.integers(1, 70), T=st.integers(6, 40), K=st.sampled_from([1, 2, 3, 8]),
       log_amp=st.floats(-1.0, 4.6), seed=st.integers(0, 2 ** 32 - 1), kernel=st.sampled_from(["hop", "three"]),
       graph=st.booleans())
def test_fuzz_stream_batch(torch_cuda, nets, S, T, K, log_amp, seed, kernel, graph):
    """S live streams fed T hops, K per call (hops_per_step), launched
    directly or as a captured hipGraph, vs the clip path on each stream's
    clip, wherever the oracle's margin on the clip's device features is
    decisive (the hop kernel runs its own FFT and an exact-f32 forward)."""
    import torch
    from vad_amd.ffn import FFNClassifier
    from vad_amd.pipeline import VadPipeline
    from vad_amd.stream import StreamBatch
    lay = nets["ref39"]
    clf = FFNClassifier(lay)
    T = (T + K - 1) // K * K
    clips = [fuzz_clip(160 * (T - 1) + 401, log_amp, seed + s, None, integral=True) for s in range(S)]
    pipe = VadPipeline(clf)
    sb = StreamBatch(S, clf, kernel=kernel, hops_per_step=K)
    sb.prime(torch.from_numpy(np.stack([c[:240] for c in clips])).cuda())
    if graph:
        sb.capture()
    hops = torch.from_numpy(np.ascontiguousarray(
        np.stack([np.stack([c[240 + 160 * t: 400 + 160 * t] for c in clips]) for t in range(T)]))).cuda()
    if K == 1:
        got = np.stack([sb.step(hops[t]).cpu().numpy().copy() for t in range(T)], axis=1)
    else:
        got = np.concatenate([sb.step_block(hops[t:t + K]).cpu().numpy().T.copy() for t in range(0, T, K)], axis=1)
    assert got.shape == (S, T)
    assert (got[:, :min(5, T)] == 255).all()
    for s, c in enumerate(clips):
        a = torch.from_numpy(c).cuda()
        want = pipe.labels(a).cpu().numpy()  # F = T frames -> T - 5 windows
        assert want.shape == (T - 5,)
        x = pipe.features(a).cpu().numpy()
        ok = O.ffn_margin(x, lay) > MARGIN_TOL
        np.testing.assert_array_equal(got[s, 5:][ok], want[ok])


@fuzz(40)
@given(depth=st.integers(1, 40), n_feat=st.sampled_from([13, 39]), n_classes=st.integers(2, 4),
       seed=st.integers(0, 2 ** 32 - 1), nan_frac=st.sampled_from([0.0, 0.05]),
       log_scale=st.floats(-4.0, 6.0))
def test_fuzz_decision_tree(torch_cuda, depth, n_feat, n_classes, seed, nan_frac, log_scale):
    """Fitted sklearn trees of random depth, width, class count and feature
    scale, trained with missing values or without: the GPU walk
    (tree_kernel.hip, thresholds rounded down to float) predicts what
    sklearn's own predict does, on fresh float32 rows with NaNs, values
    placed exactly on thresholds and their float neighbours."""
    from sklearn.tree import DecisionTreeClassifier
    from vad_amd.tree import TreeClassifier
    rng = np.random.default_rng(seed)
    scale = 10.0 ** (log_scale + rng.uniform(-1, 1, n_feat))
    X = (rng.standard_normal((3000, n_feat)) * scale).astype(np.float32)
    y = (X[:, 0] > 0).astype(int) + (X[:, 1 % n_feat] > scale[1 % n_feat]).astype(int)
    y = (y + rng.integers(0, 2, len(y))) % n_classes
    X[rng.random(X.shape) < nan_frac] = np.nan
    clf = DecisionTreeClassifier(max_depth=depth, random_state=int(seed % 1000)).fit(X, y)
    tree = TreeClassifier.from_sklearn(clf)
    Xt = (rng.standard_normal((4000, n_feat)) * scale).astype(np.float32)
    Xt[rng.random(Xt.shape) < 0.03] = np.nan
    t = clf.tree_
    # (a split that only separates missing values has an infinite threshold)
    inner = np.nonzero((t.children_left >= 0) & (np.abs(t.threshold) < 3e38))[0]
    if len(inner):  # rows sitting exactly on thresholds (as float32) and one ulp either side
        pick = rng.choice(inner, size=min(600, 3 * len(inner)))
        r = rng.integers(0, len(Xt), len(pick))
        thr = t.threshold[pick].astype(np.float32)
        delta = rng.integers(-1, 2, len(pick))
        toward = np.where(delta < 0, -np.inf, np.inf).astype(np.float32)
        Xt[r, t.feature[pick]] = np.where(delta == 0, thr, np.nextafter(thr, toward))
    np.testing.assert_array_equal(tree.predict(Xt), clf.predict(Xt))


def _spec_close(got, ref, tol=1e-5):
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    nr = np.linalg.norm(ref)
    if nr == 0:
        return np.abs(got).max() == 0
    return np.linalg.norm(got - ref) / nr <= tol


@fuzz(80)
@given(fft_n=st.one_of(st.integers(2, 8192), st.sampled_from([2, 3, 255, 256, 257, 511, 512, 513, 1024, 8192])),
       len_frac=st.floats(0.01, 2.0), log_amp=st.floats(-3.0, 4.5), seed=st.integers(0, 2 ** 32 - 1))
def test_fuzz_spec_mag_any_length(torch_cuda, fft_n, len_frac, log_amp, seed):
    """mfcc.get_spec_mag (mfcc.py:59-61) for every FFT length the reference
    accepts (2..8192; zero-padded and truncated frames): the radix-16 kernels
    at 512, a direct fp64 DFT otherwise, vs the oracle's float32 numpy FFT
    within the spectrum tolerance (1e-5 of the frame's norm)."""
    from vad_amd import mfcc as M
    rng = np.random.default_rng(seed)
    L = max(1, min(8192, int(round(len_frac * fft_n))))
    frame = (rng.standard_normal(L) * 10.0 ** log_amp).astype(np.float32)
    got = M.get_spec_mag(frame, fft_n)
    ref = O.get_spec_mag(frame, fft_n)
    assert got.shape == ref.shape == (fft_n // 2,)
    assert _spec_close(got, ref), (fft_n, L)


@fuzz(60)
@given(n=st.integers(0, 50_000), rows=st.integers(1, 4), coeff=st.floats(0.0, 1.0, exclude_max=True),
       log_amp=st.floats(-3.0, 30.0), seed=st.integers(0, 2 ** 32 - 1))
def test_fuzz_preemphasis(torch_cuda, n, rows, coeff, log_amp, seed):
    """The optional pre-emphasis stage: bit-exact to the oracle's float32
    numpy form (a rounded product, then the difference) for any length,
    coefficient and magnitude, on a clip and on each row of a frame matrix."""
    import torch
    from vad_amd.plan import preemphasis
    rng = np.random.default_rng(seed)
    x = (rng.standard_normal((rows, n)) * 10.0 ** log_amp).astype(np.float32)
    t = torch.from_numpy(np.resize(x, (rows, max(n, 1)))).cuda()[:, :n].contiguous()
    y2 = preemphasis(t, coeff).cpu().numpy()
    y1 = preemphasis(t[0].contiguous(), coeff).cpu().numpy()
    ref = np.stack([O.preemphasis(r, coeff) for r in x]) if n else np.zeros((rows, 0), np.float32)
    np.testing.assert_array_equal(y1.view(np.uint32), ref[0].view(np.uint32))
    np.testing.assert_array_equal(y2.view(np.uint32), ref.view(np.uint32))


@fuzz(40)
@given(frame_size=st.one_of(st.integers(64, 1600), st.integers(1601, 8192), st.sampled_from([513, 1025, 4097, 8192])),
       rate=st.sampled_from([8000, 16000, 22050, 44100]),
       log_amp=st.floats(-3.0, 4.5), seed=st.integers(0, 2 ** 32 - 1))
def test_fuzz_simple_features(torch_cuda, frame_size, rate, log_amp, seed):
    """SimpleAnalyser's per-frame features (simple_analyzer.py:162-215, fp64
    on the GPU) for frame sizes up to 8192 samples -- FFT lengths a power of
    two (radix-2 per wave) or one more (the reference's odd pads: a direct
    DFT) -- and any rate, vs the oracle, relative 1e-9."""
    from vad_amd.simple_analyser import SimpleAnalyser
    rng = np.random.default_rng(seed)
    sa = SimpleAnalyser(rate, frame_size, 5)
    fr = rng.standard_normal((24, frame_size)) * 10.0 ** log_amp
    fr[3] = 0.0  # a silent frame
    got = sa.frame_features(fr)
    ref = np.stack([O.simple_frame_features(f.astype(np.float32).astype(np.float64), frame_size, rate,
                                            sa.spectral_bands) for f in fr])
    np.testing.assert_allclose(got, ref, rtol=1e-9, atol=1e-9 * np.abs(ref).max())


@fuzz(60)
@given(fft_n=st.one_of(st.just(512), st.integers(64, 4096)), n_filters=st.integers(2, 64),
       mfcc_frac=st.floats(0.0, 1.0), low=st.floats(0.0, 1000.0), high_frac=st.floats(0.3, 1.0),
       sr=st.sampled_from([8000, 16000, 22050]), len_frac=st.floats(0.2, 1.5),
       log_amp=st.floats(-1.0, 4.5), seed=st.integers(0, 2 ** 32 - 1))
def test_fuzz_get_mfcc_any_bank(torch_cuda, fft_n, n_filters, mfcc_frac, low, high_frac, sr, len_frac,
                                log_amp, seed):
    """mfcc.get_mfcc (mfcc.py:67-78) with any finite mel bank the reference's
    get_mel_filterbanks builds (2..64 filters, 1..16 coefficients, any band
    and rate, FFT lengths 64..4096 and 512): the runtime-table or direct-DFT
    kernels vs the oracle within the MFCC tolerance; get_mfcc_from_spec on
    the oracle's own spectrum likewise."""
    import warnings
    from vad_amd import mfcc as M
    high = low + high_frac * (sr / 2 - low)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        fb = O.get_mel_filterbanks(low, high, fft_n, n_filters, sr)
    if not np.isfinite(fb).all() or (fb.sum(axis=1) == 0).any():
        return  # a degenerate bank (NaN rows, or filters with no bins)
    mfcc_n = 1 + int(mfcc_frac * (min(16, n_filters) - 1))
    rng = np.random.default_rng(seed)
    frame = (rng.standard_normal(max(1, int(len_frac * fft_n))) * 10.0 ** log_amp).astype(np.float32)
    got = M.get_mfcc(frame, fft_n, fb, mfcc_n)
    ref = O.get_mfcc(frame, fft_n, fb, mfcc_n)
    assert got.shape == ref.shape == (mfcc_n,)
    # the kept coefficients of the orthonormal DCT can cancel (2 filters, c0
    # only: log-energies -0.2165 and +0.2155 give c0 = -7e-4, deep run seed
    # 2323) while their rounding error scales with the log-mel row: the
    # denominators are floored at its RMS (|| full DCT || / sqrt(n_filters))
    spec = O.get_spec_mag(frame, fft_n)
    e = spec.astype(np.float64) @ fb.T
    lm = np.log10(np.where(e == 0, np.finfo(float).eps, e))
    floor = np.linalg.norm(lm) / np.sqrt(n_filters)
    assert_mfcc_close(got[None], ref[None], floor=floor)
    assert_mfcc_close(M.get_mfcc_from_spec(spec, fb, mfcc_n)[None], O.get_mfcc_from_spec(spec, fb, mfcc_n)[None],
                      floor=floor)


class _MarginRecorder:
    """Oracle-side classifier: the fp64 forward's label, recording its top-2
    margin per call (a label at a near-tie may legitimately differ)."""

    def __init__(self, layers):
        self.layers = layers
        self.margins = []

    def predict(self, x):
        x = np.asarray(x, np.float64).reshape(1, -1)
        self.margins.append(float(O.ffn_margin(x, self.layers)[0]))
        return O.ffn_labels(x, self.layers)


@fuzz(30)
@given(lens=st.lists(st.integers(1, 1500), min_size=6, max_size=40), log_amp=st.floats(0.0, 4.5),
       seed=st.integers(0, 2 ** 32 - 1), foreign=st.booleans(), silent=st.booleans())
def test_fuzz_analyser_drop_in(torch_cuda, nets, lens, log_amp, seed, foreign, silent):
    """The drop-in SKLearnAnalyzer (sklearn_analyser.py:46-82) fed frames of
    random lengths (the 512-point FFT zero-pads or truncates each), with the
    FFN in its .npz form (the fused device step) or as a pickled foreign
    classifier (device features, host predict): every call returns what the
    reference class -- restated by the oracle's AnalyserOracle -- returns
    (None, or the very frame object passed three calls earlier), wherever the
    oracle's margin for that call is decisive."""
    import pickle
    import tempfile
    from vad_amd.ffn import save_layers
    from vad_amd.sklearn_analyser import SKLearnAnalyzer
    lay = nets["ref39"]
    rng = np.random.default_rng(seed)
    frames = [(rng.standard_normal(n) * 10.0 ** log_amp).astype(np.float32) for n in lens]
    if silent:
        for i in rng.choice(len(frames), size=max(1, len(frames) // 4), replace=False):
            frames[i][:] = 0.0
    noise = [(rng.standard_normal(int(n)) * 10.0).astype(np.float32) for n in rng.integers(1, 800, 5)]
    with tempfile.TemporaryDirectory() as d:
        if foreign:
            path = f"{d}/clf.pkl"
            with open(path, "wb") as f:
                pickle.dump(O.FFNPredictor(lay), f)
        else:
            path = f"{d}/ffn.npz"
            save_layers(path, lay)
        an = SKLearnAnalyzer(path)
    rec = _MarginRecorder(lay)
    ref = O.AnalyserOracle(rec)
    for a in (an, ref):
        a.load_init_inactive_frames(noise)
    ids = {id(f): i for i, f in enumerate(frames)}
    for i, fr in enumerate(frames):
        got, want = an.feed_frame(fr), ref.feed_frame(fr)
        g = None if got is None else ids[id(got)]
        w = None if want is None else ids[id(want)]
        if i < 5:
            assert g is None and w is None
        elif rec.margins[-1] > MARGIN_TOL:
            assert g == w, (i, g, w, rec.margins[-1])


@fuzz(40)
@given(n=st.integers(1, 200_000), c=st.integers(1, 16), log_scale=st.tuples(*[st.floats(-6, 6)] * 3),
       offset=st.tuples(*[st.floats(-1e4, 1e4)] * 3), const_group=st.sampled_from([None, 0, 1, 2]),
       seed=st.integers(0, 2 ** 32 - 1))
def test_fuzz_scale_features(torch_cuda, n, c, log_scale, offset, const_group, seed):
    """scale_features (dataset/utils.py:5-34) on the device: one mean and one
    population std per group (mfcc, delta1, delta2) over every value, two
    passes in fp64 like np.std, then (x - mean) / std -- vs numpy in fp64 on
    the same float32 rows, any row count, width, scale and offset (a mean
    far from 0 with a small spread stresses the variance), a constant group
    giving numpy's inf / nan."""
    import torch
    from vad_amd import dataset as D
    rng = np.random.default_rng(seed)
    x = np.empty((n, 3, c), np.float32)
    for g in range(3):
        x[:, g] = (offset[g] + rng.standard_normal((n, c)) * 10.0 ** log_scale[g]).astype(np.float32)
    if const_group is not None:
        x[:, const_group] = np.float32(offset[const_group])
    t = torch.from_numpy(x.reshape(n, 3 * c).copy()).cuda()
    mean, std = D.scale_rows_device(t)
    a64 = x.astype(np.float64)
    m_ref = a64.mean(axis=(0, 2))
    s_ref = a64.std(axis=(0, 2))
    np.testing.assert_allclose(mean, m_ref, rtol=1e-12, atol=1e-300)
    np.testing.assert_allclose(std, s_ref, rtol=1e-9, atol=1e-12 * np.abs(m_ref).max())
    got = t.cpu().numpy().reshape(n, 3, c)
    with np.errstate(divide="ignore", invalid="ignore"):
        ref = ((a64 - mean[None, :, None]) / std[None, :, None]).astype(np.float32)
    np.testing.assert_array_equal(np.isnan(got), np.isnan(ref))
    np.testing.assert_array_equal(np.isinf(got), np.isinf(ref))
    fin = np.isfinite(ref)
    np.testing.assert_allclose(got[fin], ref[fin], rtol=3e-7, atol=3e-7 * max(1.0, np.abs(ref[fin]).max(initial=0)))


@fuzz(60)
@given(frame_len=st.one_of(st.integers(1, 1200), st.sampled_from([400, 512, 513, 800])),
       stride=st.one_of(st.integers(1, 1500), st.sampled_from([160, 400, 512])), n=st.integers(1, 300),
       nf=st.sampled_from([26, 40, 33]), fft_n=st.sampled_from([512, 512, 1024, 300]),
       log_amp=st.floats(-1.0, 4.5), seed=st.integers(0, 2 ** 32 - 1))
def test_fuzz_frame_matrix_mfcc(torch_cuda, frame_len, stride, n, nf, fft_n, log_amp, seed):
    """vad_mfcc_f32 / _i16 and vad_spec_f32 over any framing of a buffer --
    frame length 1..1200 (the FFT zero-pads or truncates), any stride
    (overlapping, abutting or with gaps), any frame count -- on the compiled
    26 / 40-filter kernels, the runtime-table kernel (33 filters) and the
    direct DFT (other FFT lengths): every frame vs the oracle; int16 input
    bit-identical to the same integer samples as fp32."""
    import torch
    from vad_amd.plan import MfccPlan
    rng = np.random.default_rng(seed)
    total = stride * (n - 1) + frame_len
    buf = np.clip(np.rint(rng.standard_normal(total) * 10.0 ** log_amp), -32767, 32767).astype(np.float32)
    fb = O.get_mel_filterbanks(300, 8000, fft_n, nf, 16000)
    if not np.isfinite(fb).all():
        return
    plan = MfccPlan(fb, 13, fft_n)
    a = torch.from_numpy(buf).cuda()
    got = plan.mfcc(a, frame_len=frame_len, frame_stride=stride, n=n).cpu().numpy()
    frames = np.stack([buf[i * stride:i * stride + frame_len] for i in range(n)])
    ref = np.stack([O.get_mfcc(f, fft_n, fb, 13) for f in frames])
    ok = mel_conditioned(frames, fft_n, fb)
    assert_mfcc_close(got[ok], ref[ok])
    got16 = plan.mfcc(a.to(torch.int16), frame_len=frame_len, frame_stride=stride, n=n).cpu().numpy()
    np.testing.assert_array_equal(got16, got)
    spec = plan.spec(a, frame_len=frame_len, frame_stride=stride, n=n).cpu().numpy()
    for i in range(n):
        assert _spec_close(spec[i], O.get_spec_mag(frames[i], fft_n)), i


@fuzz(30)
@given(frame_size=st.integers(100, 1024), hop_frac=st.floats(0.02, 1.0), nf=st.sampled_from([26, 40]),
       S=st.integers(1, 20), T=st.integers(6, 30), kernel=st.sampled_from(["hop", "three"]),
       seed=st.integers(0, 2 ** 32 - 1))
def test_fuzz_stream_configs(torch_cuda, nets, frame_size, hop_frac, nf, S, T, kernel, seed):
    """StreamBatch under any framing (frame 100..1024 samples, hop 2..100 %
    of it) and either reference bank: each stream's labels equal the clip
    path's (VadPipeline with the same MfccConfig) on that stream's samples,
    wherever the oracle's margin on the clip path's device features is
    decisive."""
    import torch
    from vad_amd.config import MfccConfig
    from vad_amd.ffn import FFNClassifier
    from vad_amd.pipeline import VadPipeline
    from vad_amd.stream import StreamBatch
    hop = max(1, int(hop_frac * frame_size))
    cfg = MfccConfig(frame_size=frame_size, hop=hop, n_filters=nf)
    lay = nets["ref39"]
    clf = FFNClassifier(lay)
    rng = np.random.default_rng(seed)
    n = hop * (T - 1) + frame_size + 1  # T frames under the strict '>' rule
    clips = np.clip(np.rint(rng.standard_normal((S, n)) * 10.0 ** rng.uniform(0, 4, (S, 1))),
                    -32767, 32767).astype(np.float32)
    keep = frame_size - hop
    sb = StreamBatch(S, clf, cfg=cfg, kernel=kernel)
    sb.prime(torch.from_numpy(np.ascontiguousarray(clips[:, :keep])).cuda())
    got = np.stack([sb.step(torch.from_numpy(np.ascontiguousarray(
        clips[:, keep + hop * t: keep + hop * (t + 1)])).cuda()).cpu().numpy().copy() for t in range(T)], axis=1)
    assert (got[:, :5] == 255).all()
    pipe = VadPipeline(clf, cfg=cfg)
    for s in range(S):
        a = torch.from_numpy(clips[s]).cuda()
        want = pipe.labels(a).cpu().numpy()
        assert want.shape == (T - 5,)
        x = pipe.features(a).cpu().numpy()
        ok = O.ffn_margin(x, lay) > MARGIN_TOL
        np.testing.assert_array_equal(got[s, 5:][ok], want[ok])


def forward_magnitude(x, lay):
    """Per row, the magnitude any rounding error of the forward scales with:
    sum |w| |h| + |b| through the layers, where a hidden unit the oracle's
    ReLU holds clearly below zero contributes nothing (it is exactly 0 on the
    device too, and ReLU is 1-Lipschitz near the kink).  A global scale instead
    wrongly excludes rows whose units all died (a width-1 hidden layer makes
    half the rows one constant logit vector; VAD_FUZZ_SEED=20261017 drew
    dims [28, 1, 22, 2] with 50 % such rows).  NaN rows: 0 (their margin is
    +inf, class 0 is checked)."""
    h = x.astype(np.float64)
    a = np.abs(h)
    for i, (W, b) in enumerate(lay):
        W, b = np.asarray(W, np.float64), np.asarray(b, np.float64)
        p, ap = h @ W + b, a @ np.abs(W) + np.abs(b)
        if i + 1 == len(lay):
            return np.nan_to_num(ap.max(axis=1), nan=0.0)
        a = np.where(p > -1e-4 * ap, ap, 0.0)
        h = np.maximum(p, 0.0)


@fuzz(50)
@given(dims=st.lists(st.integers(1, 64), min_size=2, max_size=5).map(lambda d: d[:-1] + [min(4, max(2, d[-1] % 5))]),
       arith=st.sampled_from(["split_f16", "f32"]), log_scale=st.floats(-2.0, 2.0),
       nan_rows=st.booleans(), seed=st.integers(0, 2 ** 32 - 1))
def test_fuzz_ffn_any_topology(torch_cuda, dims, arith, log_scale, nan_rows, seed):
    """FFNClassifier.predict (vad_ffn_predict) for any topology the build
    takes (1..4 layers, widths up to 64, 2..4 classes): the specialised
    split-f16 shapes where they apply, the padded exact-f32 kernel
    otherwise; rows of any scale, some NaN (class 0, np.argmax's rule):
    labels equal the fp64 oracle's wherever its top-2 margin exceeds 1e-4 of
    the logit scale."""
    from vad_amd.ffn import FFNClassifier, random_layers
    rng = np.random.default_rng(seed)
    lay = random_layers(tuple(dims), seed=int(seed % 1000))
    try:
        clf = FFNClassifier(lay, arith=arith)
        clf.plan
    except ValueError:
        assert arith == "split_f16"  # split-f16 exists for the specialised shapes only
        return
    x = (rng.standard_normal((3000, dims[0])) * 10.0 ** log_scale).astype(np.float32)
    if nan_rows:
        x[rng.random(len(x)) < 0.05, rng.integers(0, dims[0])] = np.nan
    got = clf.predict(x)
    ref = O.ffn_labels(x, lay)
    ok = O.ffn_margin(x, lay) > 1e-4 * forward_magnitude(x, lay)
    np.testing.assert_array_equal(got[ok], ref[ok])
    # non-vacuous: the bound (1e-4, ~6x a worst-case f32 / split-f16 rounding
    # of four 64-term layers) is loose for deep networks: 82-95 % of the rows
    # are checked in the deep runs' narrowest cases (dims [48, 21, 26, 2, 2],
    # [40, 1, 54, 14, 3], [2, 3, 54, 2, 4]), ~99 % typically.  A network whose
    # width-1 layers collapse every row onto a few logit vectors (dims
    # [33, 1, 1, 1, 3], deep run seed 3131: one near-tied vector) may leave
    # none to check
    z, _ = O.ffn_forward(x, lay)
    collapsed = len(np.unique(np.round(z[np.isfinite(z).all(axis=1)], 9), axis=0)) < 10
    assert collapsed or ok.mean() > 0.5


@fuzz(30)
@given(depth=st.integers(1, 30), offline=st.booleans(), F=st.integers(6, 3000),
       seed=st.integers(0, 2 ** 32 - 1))
def test_fuzz_tree_windows(torch_cuda, depth, offline, F, seed):
    """vad_features_tree (the tree over every 5-frame window, features
    computed in the kernel): labels equal sklearn's predict on the device's
    own window features (vad_features_f32), analyser (NaN windows included)
    or offline form, for trees fitted on such features."""
    import torch
    from sklearn.tree import DecisionTreeClassifier
    from vad_amd import _lib
    from vad_amd import plan as P
    from vad_amd.tree import TreeClassifier
    rng = np.random.default_rng(seed)
    clip = O.synth_clip(O.samples_for_frames(F), seed=int(seed % 10_000))
    m = P.MfccPlan(O.get_mel_filterbanks(300, 8000, 512, 26, 16000)).clip_mfcc(torch.from_numpy(clip).cuda())
    mode = _lib.FEAT_OFFLINE if offline else _lib.FEAT_ANALYSER
    x = P.window_features(m, mode).cpu().numpy()
    c0 = x[:, 0][~np.isnan(x[:, 0])]  # every window flat (all-NaN column): threshold 0
    y = rng.integers(0, 2, len(x)) ^ (np.nan_to_num(x[:, 0]) > (np.median(c0) if len(c0) else 0.0)).astype(int)
    clf = DecisionTreeClassifier(max_depth=depth, random_state=0).fit(x, y)
    tree = TreeClassifier.from_sklearn(clf)
    got = tree.window_labels(m, mode).cpu().numpy()
    np.testing.assert_array_equal(tree.classes_[got.astype(np.int64)], clf.predict(x))


@fuzz(50)
@given(L=st.integers(1, 1024), h_frac=st.floats(0.0, 1.0), S=st.integers(1, 300), fpad=st.integers(0, 70),
       hpad=st.integers(0, 70), seed=st.integers(0, 2 ** 32 - 1))
def test_fuzz_stream_push_hop(torch_cuda, L, h_frac, S, fpad, hpad, seed):
    """vad_stream_push_hop (the three-kernel form's frame assembly) for any
    frame length 1..1024, hop 1..L, padded row strides and stream count:
    every row shifted left by the hop with the new samples appended, the
    padding columns untouched."""
    import torch
    from vad_amd import _lib
    H = max(1, int(round(h_frac * L)))
    g = torch.Generator(device="cuda").manual_seed(seed)
    frames = torch.randn((S, L + fpad), device="cuda", generator=g)
    hop = torch.randn((S, H + hpad), device="cuda", generator=g)
    want = frames.clone()
    want[:, :L] = torch.cat([frames[:, H:L], hop[:, :H]], dim=1)
    _lib.check(_lib.lib().vad_stream_push_hop(_lib.ptr(frames), L + fpad, L, _lib.ptr(hop), H + hpad, H, S,
                                              _lib.stream_ptr()), "vad_stream_push_hop")
    torch.cuda.synchronize()
    assert torch.equal(frames, want)


@fuzz(50)
@given(F=st.integers(0, 400), n=st.integers(1, 16), offline=st.booleans(), flat_cols=st.integers(0, 3),
       log_scale=st.floats(-6.0, 6.0), seed=st.integers(0, 2 ** 32 - 1))
def test_fuzz_window_features_any_width(torch_cuda, F, n, offline, flat_cols, log_scale, seed):
    """vad_features_f32 over MFCC rows of any width 1..16 (the plans' MFCC
    counts) and any frame count (F - 5 windows, none below 6 frames), some
    coefficients constant (the analyser's 0/0 -> NaN in Mn and D2): the
    oracle's window features of the same fp32 rows, NaN positions exact,
    values to fp32 rounding of the window statistics."""
    import torch
    from vad_amd import _lib
    from vad_amd import plan as P
    rng = np.random.default_rng(seed)
    m = (rng.standard_normal((F, n)) * 10.0 ** log_scale).astype(np.float32)
    for c in rng.choice(n, size=min(flat_cols, n) if F else 0, replace=False):
        m[:, c] = m[0, c]
    mode = _lib.FEAT_OFFLINE if offline else _lib.FEAT_ANALYSER
    t = torch.from_numpy(np.resize(m, (max(F, 1), n))).cuda()[:F].contiguous()
    got = P.window_features(t, mode).cpu().numpy().astype(np.float64)
    rows = max(F - 5, 0)
    assert got.shape == (rows, 3 * n)
    if rows == 0:
        return
    ref = (O.offline_features(m).reshape(rows, 3 * n) if offline else O.analyser_features_fast(m))
    np.testing.assert_array_equal(np.isnan(got), np.isnan(ref))
    ok = ~np.isnan(ref)
    scale = np.abs(m).max()
    if offline:  # differences of fp32 rows: exact up to one rounding
        assert np.abs(got[ok] - ref[ok]).max() <= 4e-7 * scale
    else:  # Mn divides by the window std: its rounding scales with |M| / std
        win = np.stack([m[d:d + rows].astype(np.float64) for d in range(5)], axis=1)
        std = win.std(axis=1)
        mag = np.abs(win).max(axis=1)
        with np.errstate(divide="ignore", invalid="ignore"):
            b_mn = 4e-6 * mag / std * (1 + np.abs(np.nan_to_num(ref[:, :n]))) + 1e-6
        err = np.abs(got - ref)
        b = np.concatenate([b_mn, 4e-7 * mag + 1e-30, 2 * b_mn + 1e-6 * mag], axis=1)
        assert (err[ok] <= b[ok]).all(), float(np.max(err[ok] / b[ok]))
