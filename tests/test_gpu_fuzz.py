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
database=None: nothing is written next to the tests.
"""
import numpy as np
import pytest

from oracle import vad_oracle as O

hyp = pytest.importorskip("hypothesis")
from hypothesis import HealthCheck, given, settings  # noqa: E402
from hypothesis import strategies as st  # noqa: E402

pytestmark = pytest.mark.gpu

MFCC_TOL = 1e-4
MARGIN_TOL = 0.05
FUZZ = settings(max_examples=120, deadline=None, derandomize=True, database=None,
                suppress_health_check=[HealthCheck.function_scoped_fixture, HealthCheck.too_slow])


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


def assert_mfcc_close(got, ref):
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    assert got.shape == ref.shape
    if len(ref) == 0:
        return
    d = got - ref
    rel = np.linalg.norm(d, axis=1) / np.linalg.norm(ref, axis=1)
    mx = np.abs(d).max(axis=1) / np.abs(ref).max(axis=1)
    assert rel.max() <= MFCC_TOL, (rel.max(), int(rel.argmax()))
    assert mx.max() <= MFCC_TOL, (mx.max(), int(mx.argmax()))


@FUZZ
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
    assert_mfcc_close(mc, O.mfcc_batch(clip, fb) if F else np.zeros((0, 13)))
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


@settings(FUZZ, max_examples=50)
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
