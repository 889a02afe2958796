"""HIP path vs the oracle / reference golden vectors (needs an MI355X).

Tolerances:
  MFCC   per frame  ||d||_2 / ||ref||_2 <= 1e-4  and  max|d| <= 1e-4 * max|ref|
  spec   per frame  ||d||_2 / ||ref||_2 <= 1e-5 (float32 FFTs, different orders)
  labels bit-exact on the fixture sets (their weights are calibrated so that
         every window's fp64 top-2 logit margin exceeds 1e-3); on synthetic
         clips with random weights, bit-exact wherever the margin exceeds
         MARGIN_TOL.
"""
import pickle

import numpy as np
import pytest

from oracle import vad_oracle as O

pytestmark = pytest.mark.gpu

MFCC_TOL = 1e-4
SPEC_TOL = 1e-5
MARGIN_TOL = 0.05


def frame_rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return np.linalg.norm(a - b, axis=-1) / np.maximum(np.linalg.norm(b, axis=-1), 1e-300)


def assert_mfcc_close(got, ref):
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    assert got.shape == ref.shape
    rel = frame_rel(got, ref)
    mx = np.abs(got - ref).max(axis=-1) / np.abs(ref).max(axis=-1)
    assert rel.max() <= MFCC_TOL, (rel.max(), int(rel.argmax()))
    assert mx.max() <= MFCC_TOL, (mx.max(), int(mx.argmax()))


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    return torch


@pytest.fixture(scope="module")
def fb26():
    return O.get_mel_filterbanks(300, 8000, 512, 26, 16000)


def layers_from(w, prefix, n, b_last=None):
    lay = [(w[f"{prefix}_W{i}"], w[f"{prefix}_b{i}"]) for i in range(n)]
    if b_last is not None:
        lay[-1] = (lay[-1][0], b_last)
    return lay


# ---------------------------------------------------------------------------
# spectrum + MFCC
# ---------------------------------------------------------------------------
def test_spec_vs_reference(torch_cuda, golden, fb26):
    from vad_amd.plan import MfccPlan
    g = golden("frames")
    t = torch_cuda.from_numpy(g["frames"]).cuda()
    spec = MfccPlan(fb26).spec(t).cpu().numpy()
    ref = g["spec"]
    assert spec.dtype == np.float32 and spec.shape == ref.shape
    silent = np.linalg.norm(ref, axis=1) == 0
    assert np.all(spec[silent] == 0.0)
    assert frame_rel(spec[~silent], ref[~silent]).max() <= SPEC_TOL


@pytest.mark.parametrize("nf,key", [(26, "mfcc26"), (40, "mfcc40")])
def test_mfcc_vs_reference(torch_cuda, golden, nf, key):
    from vad_amd.plan import MfccPlan
    g = golden("frames")
    fb = O.get_mel_filterbanks(300, 8000, 512, nf, 16000)
    t = torch_cuda.from_numpy(g["frames"]).cuda()
    m = MfccPlan(fb).mfcc(t).cpu().numpy()
    assert_mfcc_close(m, g[key])
    # digital silence: c0 = log10(eps) * sqrt(n_filters) exactly as the reference
    assert abs(m[0, 0] - g[key][0, 0]) <= 1e-4 * abs(g[key][0, 0])


def test_mfcc_from_spec_vs_reference(torch_cuda, golden, fb26):
    from vad_amd.plan import MfccPlan
    g = golden("frames")
    s = torch_cuda.from_numpy(g["spec"]).cuda()
    assert_mfcc_close(MfccPlan(fb26).from_spec(s).cpu().numpy(), g["mfcc26"])


def test_spectral_null_frames(torch_cuda, golden):
    """Frames with exact spectral nulls (tests/golden/nulls.npz, made by the
    unmodified reference: cyclotomic impulse combs).  At
    the reference configuration only filter 9 of the 40-filter bank can lie
    wholly on null bins (tests/test_oracle_golden.py proves it from the
    banks), and three fixture frames null it: there the reference's energy
    is exactly 0 -> eps.  The device's spectrum is exactly 0 on every exact
    null bin (frame path, and the clip path for a one-frame clip), so its
    null filter gives the same deterministic log10(eps), and its MFCCs match
    the reference's within the MFCC rule on every frame, 26 and 40 filters."""
    torch = torch_cuda
    from vad_amd.pipeline import VadPipeline
    from vad_amd.config import MfccConfig
    from vad_amd.plan import MfccPlan
    g = golden("nulls")
    fr, nb = g["frames"], g["null_bins"]
    t = torch.from_numpy(fr).cuda()
    spec = MfccPlan(O.get_mel_filterbanks(300, 8000, 512, 26, 16000)).spec(t).cpu().numpy()
    np.testing.assert_array_equal(spec[nb], 0.0)
    assert frame_rel(spec, g["spec"]).max() <= SPEC_TOL
    fb40 = O.get_mel_filterbanks(300, 8000, 512, 40, 16000)
    null9 = nb[:, np.flatnonzero(fb40[9])].all(axis=1)
    assert null9.sum() >= 3 and ((g["spec"] @ fb40.T)[null9, 9] == 0).all()
    for nf in (26, 40):
        fb = O.get_mel_filterbanks(300, 8000, 512, nf, 16000)
        assert_mfcc_close(MfccPlan(fb).mfcc(t).cpu().numpy(), g[f"mfcc{nf}"])
        pipe = VadPipeline(cfg=MfccConfig(n_filters=nf))
        # one-frame clips: 401 samples (the reference's strict '>' framing,
        # file_processing.py:80-103, takes no frame from exactly 400)
        one = torch.cat([t, torch.zeros((len(fr), 1), device=t.device)], dim=1)
        clip = np.stack([pipe.mfcc(one[i].contiguous()).cpu().numpy()[0] for i in range(len(fr))])
        assert_mfcc_close(clip, g[f"mfcc{nf}"])


@pytest.mark.parametrize("L", [800, 512, 256, 401])
def test_other_frame_lengths(torch_cuda, golden, fb26, L):
    """np.fft.fft(x, 512) truncates frames > 512 and zero-pads short ones."""
    from vad_amd.plan import MfccPlan
    g = golden("frames")
    fr = g[f"frames_{L}"]
    p = MfccPlan(fb26)
    t = torch_cuda.from_numpy(fr).cuda()
    assert frame_rel(p.spec(t).cpu().numpy(), g[f"spec_{L}"]).max() <= SPEC_TOL
    assert_mfcc_close(p.mfcc(t).cpu().numpy(), g[f"mfcc26_{L}"])
    # odd stride / unaligned source exercises the scalar-load path
    big = np.zeros((len(fr), L + 1), np.float32)
    big[:, :L] = fr
    tb = torch_cuda.from_numpy(big.reshape(-1)).cuda()
    m2 = p.mfcc(tb, frame_len=L, frame_stride=L + 1, n=len(fr)).cpu().numpy()
    assert_mfcc_close(m2, g[f"mfcc26_{L}"])


def test_module_api_matches_reference(torch_cuda, golden, fb26):
    """vad_amd.mfcc mirrors mfcc.py: same signatures, numpy in / out."""
    from vad_amd import mfcc
    g = golden("frames")
    f = g["frames"][30]
    s = mfcc.get_spec_mag(f, 512)
    assert s.dtype == np.float32 and s.shape == (256,)
    assert frame_rel(s, g["spec"][30]) <= SPEC_TOL
    m = mfcc.get_mfcc(f, 512, fb26, 13)
    assert m.dtype == np.float64 and m.shape == (13,)
    assert_mfcc_close(m[None], g["mfcc26"][30][None])
    m2 = mfcc.get_mfcc_from_spec(g["spec"][30], fb26, 13)
    assert_mfcc_close(m2[None], g["mfcc26"][30][None])


def test_clip_mfcc_and_offline_features(torch_cuda, golden):
    """process_file on the fixture clip (file_processing.py:14-77)."""
    from vad_amd.pipeline import VadPipeline
    g = golden("clip")
    pipe = VadPipeline()
    clip = torch_cuda.from_numpy(g["clip"].astype(np.float32)).cuda()
    m = pipe.mfcc(clip).cpu().numpy()
    assert_mfcc_close(m, g["mfcc"])
    f = pipe.process_clip(g["clip"])
    ref = g["features"]
    assert f.shape == ref.shape == (93, 3, 13)
    # deltas of MFCCs: compare per row against the row's own scale
    rel = frame_rel(f.reshape(93, -1), ref.reshape(93, -1))
    assert rel.max() <= 10 * MFCC_TOL


@pytest.mark.parametrize("nf", [26, 40])
def test_int16_input_matches_fp32(torch_cuda, fb26, nf):
    """int16 PCM input (vad.py:37 astype(float32)) == the fp32 path, bitwise:
    the conversion is exact and the arithmetic after the load identical.
    Covers the compiled-table kernel (400-sample frames, aligned pairs), the
    unaligned-pair path (odd frame stride) and the spectrum entry."""
    from vad_amd.plan import MfccPlan
    torch = torch_cuda
    rng = np.random.default_rng(11)
    x16 = np.clip(O.synth_clip(160 * 4000 + 241, 5), -32768, 32767).astype(np.int16)
    x16[:2000] = rng.integers(-32768, 32767, 2000, dtype=np.int16)  # full range, incl. -32768
    fb = O.get_mel_filterbanks(300, 8000, 512, nf, 16000)
    plan = MfccPlan(fb)
    a16 = torch.from_numpy(x16).cuda()
    a32 = a16.float()
    m16 = plan.clip_mfcc(a16)
    m32 = plan.clip_mfcc(a32)
    assert torch.equal(m16, m32)
    for stride, n in ((161, 500), (160, 4000)):
        s16 = plan.spec(a16, frame_len=400, frame_stride=stride, n=n)
        s32 = plan.spec(a32, frame_len=400, frame_stride=stride, n=n)
        assert torch.equal(s16, s32)
        q16 = plan.mfcc(a16, frame_len=400, frame_stride=stride, n=n)
        q32 = plan.mfcc(a32, frame_len=400, frame_stride=stride, n=n)
        assert torch.equal(q16, q32)
    # and against the oracle on the int16 values
    ref = O.mfcc_batch(x16[: 160 * 299 + 401].astype(np.float32), fb)
    assert_mfcc_close(m16[:300].cpu().numpy(), ref)


def test_int16_labels_match_fp32(torch_cuda, golden):
    """VadPipeline.labels on int16 PCM (vad_mfcc_ffn_i16) == on the same
    samples as float32 (vad_mfcc_ffn), for the FFN and the decision tree."""
    from vad_amd.ffn import FFNClassifier
    from vad_amd.pipeline import VadPipeline
    torch = torch_cuda
    w = golden("ffn")
    x16 = np.clip(O.synth_clip(160 * 6000 + 241, 9), -32768, 32767).astype(np.int16)
    a16 = torch.from_numpy(x16).cuda()
    for clf in (FFNClassifier(layers_from(w, "ref39", 4)), _tree(golden)[1]):
        pipe = VadPipeline(clf)
        assert torch.equal(pipe.labels(a16), pipe.labels(a16.float()))
    with pytest.raises(TypeError):
        VadPipeline(FFNClassifier(layers_from(w, "ref39", 4))).labels(a16.double())


def test_framing_edge_lengths(torch_cuda, fb26):
    from vad_amd.pipeline import VadPipeline
    pipe = VadPipeline()
    for L in (0, 1, 400, 401, 560, 561, 1200):
        a = torch_cuda.from_numpy(O.synth_clip(max(L, 1), 3)[:L].copy()).cuda()
        if L == 0:
            a = torch_cuda.zeros(0, device="cuda")
        m = pipe.mfcc(a).cpu().numpy()
        assert m.shape == (O.n_frames(L), 13)
        if len(m):
            assert_mfcc_close(m, O.mfcc_batch(a.cpu().numpy(), fb26))


# ---------------------------------------------------------------------------
# features + FFN labels
# ---------------------------------------------------------------------------
def test_ffn_predict_bit_exact(torch_cuda, golden):
    """fp32 MFMA forward vs the fp64 oracle on the fixture feature rows."""
    from vad_amd.ffn import FFNClassifier
    w = golden("ffn")
    x = w["test_x"]
    for prefix, n, key, dim in (("ref39", 4, "test_labels_ref39", 39),
                                ("bl13", 3, "test_labels_bl13", 13)):
        clf = FFNClassifier(layers_from(w, prefix, n))
        got = clf.predict(x[:, :dim])
        np.testing.assert_array_equal(got, w[key])
    # NaN rows (constant windows) -> class 0
    assert np.isnan(x).any(axis=1).sum() > 0


def test_ffn_generic_topology(torch_cuda):
    """A shape outside the specialised ones runs on the padded generic kernel."""
    from vad_amd.ffn import FFNClassifier, random_layers
    rng = np.random.default_rng(4)
    for dims in ((20, 48, 3), (39, 4), (7, 33, 17, 5, 4), (64, 64, 64, 64, 2)):
        lay = random_layers(dims, seed=len(dims))
        x = rng.standard_normal((333, dims[0])) * 2
        ref = O.ffn_labels(x.astype(np.float32), lay)
        marg = O.ffn_margin(x.astype(np.float32), lay)
        got = FFNClassifier(lay).predict(x)
        ok = marg > 1e-4
        np.testing.assert_array_equal(got[ok], ref[ok])


def test_ffn_split_f16_rescale(torch_cuda, golden):
    """Window labels of networks whose activations overflow f16: the split-f16
    MFMA path reruns such tiles at a power-of-two scale.  Scaling layer l's
    weights by 2^10 and its bias by 2^(10 (l + 1)) scales every activation by
    a power of two, so the labels are the unscaled network's.  bl13 at 2^16
    also takes its layer-1 check (the host's analyser bound on the layer-1
    inputs, FfnDev::h1_bounded, exceeds 32768 there; at 2^10 the bound holds
    and the check is skipped)."""
    from vad_amd.ffn import FFNClassifier
    from vad_amd.pipeline import VadPipeline
    w = golden("ffn")
    clip = torch_cuda.from_numpy(w["test_clip"]).cuda()
    m = VadPipeline().mfcc(clip)
    for prefix, n, e in (("ref39", 4, 10), ("bl13", 3, 10), ("bl13", 3, 16)):
        lay = [(W * 2.0 ** e, b * 2.0 ** (e * (i + 1)))
               for i, (W, b) in enumerate(layers_from(w, prefix, n))]
        got = FFNClassifier(lay).plan.window_labels(m).cpu().numpy()
        sure = w[f"test_margin_{prefix}"] > MARGIN_TOL
        np.testing.assert_array_equal(got[sure], w[f"test_labels_{prefix}"][sure])


def test_ffn_label_difference_overflowed_logits(torch_cuda):
    """The labels-only launches of a 13-64-64-2 network decide by the logit
    difference d = z1 - z0 (ffn_dev.h valu_label2) and rerun a wave's 16
    windows (tile t: windows 16 t .. 16 t + 15) in the two-logit form when
    some d is not finite.  Scaling layer 1 by 2^16 and the output layer by
    2^112 (every weight within f16 / f32 range) pushes many windows' f32
    logits past 2^128:
      * output columns mixed 0.95 / 0.05 (correlated logits, small
        difference weights): in tiles where no partial sum of d can overflow
        (sum_k |fd_k h_k| < 2^127.5, fp64), the labels are the fp64 oracle's
        (the sign of z1 - z0) even where the f32 logits are infinite -- where
        argmax of the two-logit form is arbitrary (an overflowed partial sum
        of z0 can even give +inf for a negative exact z0);
      * unmixed: in tiles where some |d| exceeds 1.01 * 2^128 (d overflows
        in any f32 order), every window carries the logits launch's label
        (vad_features_ffn_logits: the same two-logit code and argmax rules);
      * finite logits apart from f32 near-ties: both launches agree;
        NaN-flagged windows are class 0; the fused kernel agrees with both
        there."""
    from vad_amd import plan as P
    from vad_amd.ffn import TOPOLOGY_BL13, FFNClassifier, random_layers
    from vad_amd.pipeline import VadPipeline
    F = 20000
    clip = O.synth_clip(160 * (F - 1) + 401, seed=11).astype(np.float32)
    a = torch_cuda.from_numpy(clip).cuda()
    m = VadPipeline().mfcc(a)
    x = P.window_features(m, 0).cpu().numpy()[:, :13].astype(np.float64)
    flag = np.isnan(x).any(axis=1)
    nt = (len(x) + 15) // 16

    def per_tile_max(v):
        p = np.zeros(nt * 16)
        p[:len(v)] = np.nan_to_num(np.where(flag, 0.0, v))
        return np.repeat(p.reshape(nt, 16).max(axis=1), 16)[:len(v)]

    for mix in (0.95, 0.0):
        lay = random_layers(TOPOLOGY_BL13, seed=5)
        W, b = lay[-1]
        W = W.copy()
        W[:, 1] = mix * W[:, 0] + (1 - mix) * W[:, 1]
        lay = lay[:-1] + [(W, b)]
        lay_s = [lay[0], tuple((t * 2.0 ** 16).astype(np.float32) for t in lay[1]),
                 tuple((t * 2.0 ** 112).astype(np.float32) for t in lay[2])]
        clf = FFNClassifier(lay_s)
        lab = clf.plan.window_labels(m).cpu().numpy()
        lab_l, zl = (t.cpu().numpy() for t in P.window_logits(clf.plan, m))
        # the logits launch takes its labels from the same difference: a
        # label never depends on whether the logits were requested
        np.testing.assert_array_equal(lab, lab_l)
        np.testing.assert_array_equal(lab[flag], 0)
        # fp64 hidden activations of the scaled network, and the device's f32
        # difference weights (class 1 minus class 0 of the f32 plan weights)
        h = x
        for Wl, bl in lay_s[:2]:
            h = O.relu_keep_nan(h @ Wl.astype(np.float64) + bl.astype(np.float64))
        W2, b2 = lay_s[2]
        fd = (W2[:, 1] - W2[:, 0]).astype(np.float64)
        d64 = h @ fd + float(b2[1] - b2[0])
        quiet = per_tile_max(np.abs(h) @ np.abs(fd)) < 2.0 ** 127.5
        rerun = per_tile_max(np.abs(d64)) > 1.01 * 2.0 ** 128
        big = ~np.isfinite(zl).all(axis=1) & ~flag
        with np.errstate(over="ignore", invalid="ignore"):
            fin = np.isfinite(zl).all(axis=1) & ~flag
            rel = fin & (np.abs(zl[:, 1] - zl[:, 0]) > 1e-5 * np.abs(zl).max(axis=1))
        np.testing.assert_array_equal(lab[rel], lab_l[rel])
        sure = np.abs(d64) > 1e-5 * np.abs(h @ W2.astype(np.float64)).max(axis=1)
        ref = (d64 > 0).astype(np.uint8)  # argmax of two finite fp64 logits
        sel = quiet & sure & ~flag
        np.testing.assert_array_equal(lab[sel], ref[sel])
        np.testing.assert_array_equal(lab[rerun], lab_l[rerun])
        if mix == 0.95:
            assert (sel & big).sum() > 1000, int((sel & big).sum())
        else:
            assert (rerun & big).sum() > 1000, int((rerun & big).sum())
        # the fused kernel (its own tiles) on bit-identical MFCC rows
        lab_f = VadPipeline(clf).labels(a, fused=True).cpu().numpy()
        det = flag | rel
        np.testing.assert_array_equal(lab_f[det], lab[det])


def test_window_labels_random_nets_long_clip(torch_cuda):
    """Window labels of both specialised topologies (split-f16 MFMA path; a
    3-class 13-64-64-3 runs the bl13 shape with its fragments in LDS) on a
    20k-frame synthetic clip with digital silence (NaN windows) vs the
    oracle's forward on the same device features, where the oracle's top-2
    margin exceeds 1e-3."""
    from vad_amd import plan as P
    from vad_amd.ffn import TOPOLOGY_BL13, TOPOLOGY_REF39, FFNClassifier, random_layers
    from vad_amd.pipeline import VadPipeline
    F = 20000
    clip = O.synth_clip(160 * (F - 1) + 401, seed=7).astype(np.float32)
    for topo in (TOPOLOGY_BL13, TOPOLOGY_REF39, (13, 64, 64, 3)):
        lay = random_layers(topo, seed=3)
        pipe = VadPipeline(FFNClassifier(lay))
        m = pipe.mfcc(torch_cuda.from_numpy(clip).cuda())
        got = pipe.ffn.plan.window_labels(m).cpu().numpy()
        x = P.window_features(m, 0).cpu().numpy()[:, :topo[0]]
        ref = O.ffn_labels(x, lay)
        ok = O.ffn_margin(x, lay) > 1e-3
        assert np.isnan(x).any(axis=1).sum() > 0  # NaN windows are exercised
        np.testing.assert_array_equal(got[ok], ref[ok])
        assert ok.mean() > 0.99


def test_analyser_features_and_labels_on_clip(torch_cuda, golden, fb26):
    """Whole-clip analyser windows: GPU features/labels vs the oracle."""
    from vad_amd import plan as P
    from vad_amd.ffn import FFNClassifier
    from vad_amd.pipeline import VadPipeline
    w = golden("ffn")
    clf = FFNClassifier(layers_from(w, "ref39", 4))
    pipe = VadPipeline(clf)
    clip = torch_cuda.from_numpy(w["test_clip"]).cuda()
    feats = pipe.features(clip).cpu().numpy().astype(np.float64)
    ref = w["test_x"]
    nan_rows = np.isnan(ref).any(axis=1)
    np.testing.assert_array_equal(np.isnan(feats).any(axis=1), nan_rows)
    labels = pipe.labels(clip).cpu().numpy()
    ref_l = w["test_labels_ref39"]
    marg = w["test_margin_ref39"]
    sure = marg > MARGIN_TOL
    np.testing.assert_array_equal(labels[sure], ref_l[sure])
    # every fixture window's margin exceeds 1e-3 (gen_golden calibrates the
    # weights for it): the labels are exact, not just above MARGIN_TOL
    assert marg.min() > 1e-3
    np.testing.assert_array_equal(labels, ref_l)
    # same labels from the two-step device path
    m = pipe.mfcc(clip)
    np.testing.assert_array_equal(clf.plan.window_labels(m).cpu().numpy(), labels)
    # offline features on device equal the host-visible process_clip rows
    off = P.window_features(m, 1).cpu().numpy()
    assert off.shape == (len(ref_l), 39)


def test_labels_short_clips(torch_cuda, golden):
    from vad_amd.ffn import FFNClassifier
    from vad_amd.pipeline import VadPipeline
    w = golden("ffn")
    pipe = VadPipeline(FFNClassifier(layers_from(w, "ref39", 4)))
    for L in (0, 400, 1041, 1200, 1201):
        a = torch_cuda.zeros(max(L, 1), device="cuda")[:L].contiguous()
        lab = pipe.labels(a)
        assert lab.numel() == max(O.n_frames(L) - 5, 0)


# ---------------------------------------------------------------------------
# drop-in analyser (feed_frame) traces
# ---------------------------------------------------------------------------
def _save_weights(tmp_path, w, b_last=None):
    from vad_amd.ffn import save_layers
    p = tmp_path / "ffn.npz"
    save_layers(str(p), layers_from(w, "ref39", 4, b_last))
    return str(p)


def _replay(an, stream):
    rets = []
    for f in stream:
        r = an.feed_frame(f)
        rets.append(-1 if r is None else next(i for i, s in enumerate(stream) if s is r))
    return np.asarray(rets)


def test_analyser_trace_matches_reference(torch_cuda, golden, tmp_path):
    from vad_amd.sklearn_analyser import SKLearnAnalyzer
    g = golden("analyser")
    w = golden("ffn")
    an = SKLearnAnalyzer(_save_weights(tmp_path, w), fft_n=512)
    an.load_init_inactive_frames(list(g["noise"]))
    stream = list(g["stream"])
    rets = _replay(an, stream)
    ref = g["returns"]
    # oracle margins of the windows this trace classified
    marg = O.ffn_margin(g["features"], layers_from(w, "ref39", 4))
    sure = np.concatenate([np.ones(5, bool), marg > MARGIN_TOL])
    np.testing.assert_array_equal(rets[sure], ref[sure])
    assert marg.min() > 1e-3  # calibrated fixture: every classified window is decisive
    np.testing.assert_array_equal(rets, ref)


def test_analyser_blocks_and_errors(torch_cuda, golden, tmp_path):
    from vad_amd.sklearn_analyser import SKLearnAnalyzer
    g = golden("analyser")
    w = golden("ffn")
    path = _save_weights(tmp_path, w)
    an = SKLearnAnalyzer(path)
    an.load_init_inactive_frames(list(g["noise"]))
    blocks = list(g["blocks"])  # vad.py's 800-value blocks: truncated to 512
    np.testing.assert_array_equal(_replay(an, blocks), g["returns_blocks"])
    # no load_init_inactive_frames -> TypeError on the first feed_frame
    an2 = SKLearnAnalyzer(path)
    with pytest.raises(TypeError):
        an2.feed_frame(g["stream"][0])
    with pytest.raises(ValueError):
        an2.load_init_inactive_frames(list(g["noise"][:4]))
    # MUSIC-capable weights: AssertionError at the same call as the reference
    an3 = SKLearnAnalyzer(_save_weights(tmp_path, w, w["ref39_b3_music"]))
    an3.load_init_inactive_frames(list(g["noise"]))
    k = int(str(g["error_music"]).split(":")[0])
    stream = list(g["stream"])
    rets = [an3.feed_frame(f) for f in stream[:k]]
    ref = g["returns_music"]
    assert [(-1 if r is None else next(i for i, s in enumerate(stream) if s is r)) for r in rets] \
        == list(ref)
    with pytest.raises(AssertionError):
        an3.feed_frame(stream[k])


class _Recorder:
    """A foreign (non-FFN) classifier: records the rows the analyser passes."""

    def __init__(self, labels):
        self.labels = list(labels)
        self.rows = []

    def predict(self, x):
        self.rows.append(np.array(x))
        return np.array([self.labels[len(self.rows) - 1]])


def test_analyser_foreign_classifier(torch_cuda, golden, tmp_path):
    from vad_amd.sklearn_analyser import SKLearnAnalyzer
    g = golden("analyser")
    ref_rows = g["features"]
    w = golden("ffn")
    labels = O.ffn_labels(ref_rows, layers_from(w, "ref39", 4))
    p = tmp_path / "clf.pkl"
    with open(p, "wb") as f:
        pickle.dump(_Recorder(labels), f)
    an = SKLearnAnalyzer(str(p))
    an.load_init_inactive_frames(list(g["noise"]))
    rets = _replay(an, list(g["stream"]))
    np.testing.assert_array_equal(rets, g["returns"])
    rows = np.concatenate(an.classifier.rows)
    assert rows.dtype == np.float64 and rows.shape == ref_rows.shape
    nan_rows = np.isnan(ref_rows).any(axis=1)
    np.testing.assert_array_equal(np.isnan(rows).any(axis=1), nan_rows)


# ---------------------------------------------------------------------------
# streaming batch (config 5) == clip path
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("S", [1, 5, 24])  # hop kernel blocks hold >= 4 streams: partial blocks too
def test_stream_batch_matches_clip_path(torch_cuda, golden, S):
    from vad_amd.ffn import FFNClassifier
    from vad_amd.pipeline import VadPipeline
    from vad_amd.stream import StreamBatch
    w = golden("ffn")
    clf = FFNClassifier(layers_from(w, "ref39", 4))
    T = 40
    clips = [O.synth_clip(160 * (T - 1) + 401, seed=600 + s) for s in range(S)]
    pipe = VadPipeline(clf)
    want = np.stack([pipe.labels(torch_cuda.from_numpy(c).cuda()).cpu().numpy() for c in clips])
    fb = O.get_mel_filterbanks(300, 8000, 512, 26, 16000)
    marg = np.stack([O.ffn_margin(O.analyser_features_fast(O.mfcc_batch(c, fb)), layers_from(w, "ref39", 4))
                     for c in clips])
    for kernel, use_graph in (("three", False), ("three", True), ("hop", False), ("hop", True)):
        sb = StreamBatch(S, clf, kernel=kernel)
        sb.prime(torch_cuda.from_numpy(np.stack([c[:240] for c in clips])).cuda())
        if use_graph:
            sb.capture()
        got = []
        for t in range(T):
            new = np.stack([c[240 + 160 * t: 400 + 160 * t] for c in clips])
            got.append(sb.step(torch_cuda.from_numpy(new).cuda()).cpu().numpy().copy())
        got = np.stack(got, axis=1)  # (S, T)
        assert (got[:, :5] == 255).all()
        if kernel == "three":  # the clip path's own MFCC kernel: identical labels
            np.testing.assert_array_equal(got[:, 5:], want[:, :T - 5])
        else:  # its own FFT and f32 VALU forward: identical wherever the label is decisive
            ok = marg > 1e-3
            np.testing.assert_array_equal(got[:, 5:][ok], want[:, :T - 5][ok])


@pytest.mark.parametrize("topo", [(13, 64, 64, 2), (13, 64, 64, 3)])
def test_stream_hop_narrow_networks(torch_cuda, topo):
    """The one-kernel hop with a network that takes only the 13 normalised
    coefficients (layer 0 reads its inputs in fours: columns 13..15 must be
    zeros, not D1[0..2]): labels vs the oracle on x[:, :13] of each stream's
    features, wherever the oracle's top-2 margin exceeds 1e-3."""
    from vad_amd.ffn import FFNClassifier, random_layers
    from vad_amd.stream import StreamBatch
    S, T = 8, 40
    layers = random_layers(topo, seed=11)
    clips = [O.synth_clip(160 * (T - 1) + 401, seed=700 + s) for s in range(S)]
    fb = O.get_mel_filterbanks(300, 8000, 512, 26, 16000)
    sb = StreamBatch(S, FFNClassifier(layers), kernel="hop")
    sb.prime(torch_cuda.from_numpy(np.stack([c[:240] for c in clips])).cuda())
    got = []
    for t in range(T):
        new = np.stack([c[240 + 160 * t: 400 + 160 * t] for c in clips])
        got.append(sb.step(torch_cuda.from_numpy(new).cuda()).cpu().numpy().copy())
    got = np.stack(got, axis=1)[:, 5:]  # (S, T-5)
    n_ok = 0
    for s, c in enumerate(clips):
        x = O.analyser_features_fast(O.mfcc_batch(c, fb))[:, :13]
        ok = O.ffn_margin(x, layers) > 1e-3
        np.testing.assert_array_equal(got[s][ok], O.ffn_labels(x, layers)[ok])
        n_ok += int(ok.sum())
    assert n_ok > 0.95 * got.size
    assert len(np.unique(got)) >= 2


@pytest.mark.parametrize("kernel,K", [("hop", 2), ("hop", 8), ("three", 3)])
def test_stream_hop_blocks_equal_single_hops(torch_cuda, golden, kernel, K):
    """K hops per step (vad_stream_hops: one launch; the three-kernel form: K
    pushes + steps), launched directly and as a captured hipGraph reading its
    static input block in place: labels, frames, ring and counts identical to
    K single-hop steps."""
    import torch
    from vad_amd.ffn import FFNClassifier
    from vad_amd.stream import StreamBatch
    w = golden("ffn")
    clf = FFNClassifier(layers_from(w, "ref39", 4))
    S, nb = 24, 6
    T = K * nb
    clips = [O.synth_clip(160 * (T - 1) + 401, seed=800 + s) for s in range(S)]
    carry = torch.from_numpy(np.stack([c[:240] for c in clips])).cuda()
    hops = torch.from_numpy(np.ascontiguousarray(
        np.stack([np.stack([c[240 + 160 * t: 400 + 160 * t] for c in clips]) for t in range(T)]))).cuda()
    ref = StreamBatch(S, clf, kernel=kernel)
    ref.prime(carry)
    want = torch.stack([ref.step(hops[t]).clone() for t in range(T)])  # (T, S)
    for graph in (False, True):
        sb = StreamBatch(S, clf, kernel=kernel, hops_per_step=K)
        sb.prime(carry)
        if graph:
            sb.capture()
        got = []
        for b in range(nb):
            blk = hops[b * K:(b + 1) * K]
            if graph:
                sb.inputs.copy_(blk)  # the producer's write into the static block
                got.append(sb.step_block().clone())
            else:
                got.append(sb.step_block(blk).clone())
        got = torch.cat(got)
        assert torch.equal(got, want), (graph, int((got != want).sum()))
        assert torch.equal(sb.frames, ref.frames) and torch.equal(sb.ring, ref.ring)
        assert torch.equal(sb.count, ref.count)
    assert (want[:5] == 255).all() and (want[5:] != 255).all()


def test_stream_hop_block_stream_major(torch_cuda, golden):
    """A block in stream-major order -- each stream's K hops contiguous, an
    (S, K * hop) buffer viewed as (K, S, hop): block stride hop, row stride
    K * hop -- is read in place by vad_stream_hops (disjoint rows, the other
    ordering) and gives the labels and state of K single-hop steps; a view
    whose rows overlap falls back to a copy in step_block."""
    import torch
    from vad_amd import _lib
    from vad_amd.ffn import FFNClassifier
    from vad_amd.stream import StreamBatch, hop_rows_disjoint
    w = golden("ffn")
    clf = FFNClassifier(layers_from(w, "ref39", 4))
    S, K, nb = 24, 8, 3
    T = K * nb
    clips = [O.synth_clip(160 * (T - 1) + 401, seed=850 + s) for s in range(S)]
    carry = torch.from_numpy(np.stack([c[:240] for c in clips])).cuda()
    per_stream = torch.from_numpy(np.stack([c[240:240 + 160 * T] for c in clips])).cuda()  # (S, T*hop)
    ref = StreamBatch(S, clf)
    ref.prime(carry)
    want = torch.stack([ref.step(per_stream[:, 160 * t:160 * (t + 1)].contiguous()).clone() for t in range(T)])
    sb = StreamBatch(S, clf, hops_per_step=K)
    sb.prime(carry)
    got = []
    for b in range(nb):
        blk = per_stream[:, 160 * K * b:160 * K * (b + 1)].contiguous().view(S, K, 160).transpose(0, 1)
        assert blk.stride() == (160, K * 160, 1) and hop_rows_disjoint(S, K, 160, K * 160, 160)
        got.append(sb.step_block(blk).clone())
    got = torch.cat(got)
    assert torch.equal(got, want), int((got != want).sum())
    assert torch.equal(sb.frames, ref.frames) and torch.equal(sb.ring, ref.ring)
    # the C ABI itself accepts that layout (rc 0) and refuses an overlapping one
    L = _lib.lib()
    ok = per_stream[:, :160 * K].contiguous()
    rc = L.vad_stream_hops(sb.plan.handle, sb.ffn.plan.handle, _lib.ptr(sb.frames), 400, 400, _lib.ptr(ok),
                           K * 160, 160, S, K, 160, _lib.ptr(sb.ring), _lib.ptr(sb.count),
                           _lib.ptr(sb.label_block), S, _lib.stream_ptr())
    assert rc == 0
    rc = L.vad_stream_hops(sb.plan.handle, sb.ffn.plan.handle, _lib.ptr(sb.frames), 400, 400, _lib.ptr(ok),
                           K * 160 - 1, 160, S, K, 160, _lib.ptr(sb.ring), _lib.ptr(sb.count),
                           _lib.ptr(sb.label_block), S, _lib.stream_ptr())
    assert rc == _lib.VAD_EINVAL
    torch.cuda.synchronize()


@pytest.mark.parametrize("K,graph", [(1, False), (1, True), (8, False), (8, True)])
def test_stream_host_io_steps(torch_cuda, golden, K, graph):
    """C5 as SURVEY 8(d) times it: each step copies every stream's new
    samples from pinned host memory, runs the hop kernel and copies the
    labels back (step_host; captured into the hipGraph with host_io=True and
    replayed through vad_graph_launch): the host labels equal the
    device-input single-hop steps', and the state ends identical."""
    import torch
    from vad_amd.ffn import FFNClassifier
    from vad_amd.stream import StreamBatch
    w = golden("ffn")
    clf = FFNClassifier(layers_from(w, "ref39", 4))
    S, nb = 512, 4
    T = K * nb
    clips = np.stack([O.synth_clip(160 * (T - 1) + 401, seed=900 + s) for s in range(S)])
    carry = torch.from_numpy(np.ascontiguousarray(clips[:, :240])).cuda()
    hops = np.ascontiguousarray(np.stack([clips[:, 240 + 160 * t: 400 + 160 * t] for t in range(T)]))
    ref = StreamBatch(S, clf)
    ref.prime(carry)
    want = torch.stack([ref.step(torch.from_numpy(hops[t]).cuda()).clone() for t in range(T)]).cpu()
    sb = StreamBatch(S, clf, hops_per_step=K)
    sb.prime(carry)
    if graph:
        sb.capture(host_io=True)
    else:
        sb.attach_host_io()
    got = []
    for b in range(nb):
        sb.host_inputs.copy_(torch.from_numpy(hops[b * K:(b + 1) * K]))
        lab = sb.step_host()
        torch.cuda.current_stream().synchronize()
        got.append(lab.clone())
    got = torch.cat(got)
    assert torch.equal(got, want), int((got != want).sum())
    assert torch.equal(sb.frames, ref.frames) and torch.equal(sb.ring, ref.ring)
    assert (want[5:] != 255).all()


def test_stream_hops_rejects_overlapping_blocks(torch_cuda, golden):
    """vad_stream_hops refuses hop blocks that repeat or overlap (a zero or
    short hop_block_stride with n_hops > 1) before launching anything."""
    import ctypes
    import torch
    from vad_amd import _lib
    from vad_amd.ffn import FFNClassifier
    from vad_amd.stream import StreamBatch
    w = golden("ffn")
    sb = StreamBatch(4, FFNClassifier(layers_from(w, "ref39", 4)), hops_per_step=2)
    L = _lib.lib()
    for bs in (0, -640, 3 * 160):
        rc = L.vad_stream_hops(sb.plan.handle, sb.ffn.plan.handle, _lib.ptr(sb.frames), 400, 400,
                               _lib.ptr(sb.inputs), 160, 160, 4, 2, bs, _lib.ptr(sb.ring), _lib.ptr(sb.count),
                               _lib.ptr(sb.label_block), 4, _lib.stream_ptr())
        assert rc == _lib.VAD_EINVAL, (bs, rc)
    assert (sb.count == 0).all()  # nothing ran


@pytest.mark.parametrize("frame_size,hop,nf", [(512, 256, 26), (1000, 400, 26), (400, 160, 40)])
def test_stream_hop_long_frames(torch_cuda, golden, frame_size, hop, nf):
    """Frames longer than 448 samples take the hop kernel's 16-chunk build
    (stream_kernel.hip, NR = 16; 1000 samples: the FFT truncates to 512, as
    np.fft.fft(x, 512) does), and 40 filters take 40 mel lanes: the MFCC
    ring matches the three-kernel form's (the clip MFCC kernel on the same
    frames) to 1e-4 per row, blocks of hops equal single hops, and the
    labels agree wherever both rings do."""
    import torch
    from vad_amd.config import MfccConfig
    from vad_amd.ffn import FFNClassifier
    from vad_amd.stream import StreamBatch
    w = golden("ffn")
    clf = FFNClassifier(layers_from(w, "ref39", 4))
    cfg = MfccConfig(frame_size=frame_size, hop=hop, n_filters=nf)
    S, T, K = 5, 16, 4
    carry_n = frame_size - hop
    clips = [O.synth_clip(hop * T + carry_n, seed=900 + s) for s in range(S)]
    carry = torch.from_numpy(np.stack([c[:carry_n] for c in clips])).cuda()
    hops = torch.from_numpy(np.ascontiguousarray(np.stack(
        [np.stack([c[carry_n + hop * t: carry_n + hop * (t + 1)] for c in clips]) for t in range(T)]))).cuda()
    three = StreamBatch(S, clf, cfg=cfg, kernel="three")
    one = StreamBatch(S, clf, cfg=cfg, kernel="hop")
    three.prime(carry)
    one.prime(carry)
    lab3, lab1 = [], []
    for t in range(T):
        lab3.append(three.step(hops[t]).clone())
        lab1.append(one.step(hops[t]).clone())
        a, b = one.ring.double().cpu().numpy(), three.ring.double().cpu().numpy()
        rel = np.linalg.norm(a - b, axis=2) / np.maximum(np.linalg.norm(b, axis=2), 1e-30)
        assert rel.max() <= 1e-4, (t, rel.max())
    assert torch.equal(one.frames, three.frames)
    assert torch.equal(one.count, three.count)
    blk = StreamBatch(S, clf, cfg=cfg, kernel="hop", hops_per_step=K)
    blk.prime(carry)
    got = torch.cat([blk.step_block(hops[b * K:(b + 1) * K]).clone() for b in range(T // K)])
    assert torch.equal(got, torch.stack(lab1))
    assert torch.equal(blk.ring, one.ring) and torch.equal(blk.frames, one.frames)
    same = (torch.stack(lab1) == torch.stack(lab3)).float().mean().item()
    assert same >= 0.9, same


def test_stream_hop_rejects_window(torch_cuda):
    """An analysis-window plan cannot run the one-kernel hop (its table blob
    has no window): StreamBatch refuses it, and so does the C ABI."""
    import torch
    from vad_amd import _lib
    from vad_amd.config import MfccConfig
    from vad_amd.ffn import FFNClassifier, random_layers
    from vad_amd.plan import MfccPlan
    from vad_amd.stream import StreamBatch
    clf = FFNClassifier(random_layers((39, 64, 32, 16, 3), seed=1))
    cfg = MfccConfig(window="hamming")
    with pytest.raises(ValueError):
        StreamBatch(2, clf, cfg=cfg, kernel="hop")
    StreamBatch(2, clf, cfg=cfg, kernel="three")  # the three-kernel form applies it
    plan = MfccPlan.from_config(cfg)
    S = 2
    frames = torch.zeros((S, 400), device="cuda")
    hop = torch.zeros((S, 160), device="cuda")
    ring = torch.zeros((S, 5, 13), device="cuda")
    count = torch.zeros((S,), dtype=torch.int32, device="cuda")
    labels = torch.zeros((S,), dtype=torch.uint8, device="cuda")
    rc = _lib.lib().vad_stream_hop(plan.handle, clf.plan.handle, _lib.ptr(frames), 400, 400, _lib.ptr(hop), 160,
                                   160, S, _lib.ptr(ring), _lib.ptr(count), _lib.ptr(labels), _lib.stream_ptr())
    assert rc == _lib.VAD_EUNSUPPORTED


@pytest.mark.parametrize("L,H", [(400, 160), (400, 400), (600, 1), (1024, 160)])
def test_stream_push_hop(torch_cuda, L, H):
    """vad_stream_push_hop == shift left by H and append the new samples."""
    import torch
    from vad_amd import _lib
    S = 37
    g = torch.Generator(device="cuda").manual_seed(L + H)
    frames = torch.randn((S, L + 3), device="cuda", generator=g)  # row stride L + 3
    hop = torch.randn((S, H + 2), device="cuda", generator=g)
    want = frames.clone()
    want[:, :L] = torch.cat([frames[:, H:L], hop[:, :H]], dim=1)
    _lib.check(_lib.lib().vad_stream_push_hop(_lib.ptr(frames), L + 3, L, _lib.ptr(hop), H + 2, H, S,
                                              _lib.stream_ptr()), "vad_stream_push_hop")
    torch.cuda.synchronize()
    assert torch.equal(frames, want)
    assert _lib.lib().vad_stream_push_hop(_lib.ptr(frames), L + 3, L, _lib.ptr(hop), H + 2, L + 1, S,
                                          _lib.stream_ptr()) == _lib.VAD_EINVAL


# ---------------------------------------------------------------------------
# full-size properties (BASELINE config 3 size)
# ---------------------------------------------------------------------------
def test_full_size_properties(torch_cuda, golden):
    import torch
    from vad_amd.ffn import FFNClassifier
    from vad_amd.pipeline import VadPipeline
    w = golden("ffn")
    pipe = VadPipeline(FFNClassifier(layers_from(w, "ref39", 4)))
    F = 1_000_000
    L = 160 * (F - 1) + 401
    g = torch.Generator(device="cuda").manual_seed(1)
    audio = torch.randn(L, device="cuda", generator=g) * 1000.0
    audio[5_000_000:5_100_000] = 0.0  # a silent stretch
    lab1 = pipe.labels(audio)
    lab2 = pipe.labels(audio)
    assert lab1.numel() == F - 5
    assert torch.equal(lab1, lab2)                      # deterministic
    assert int(lab1.max()) <= 2
    # a segment cut at a frame boundary with a 240-sample + 4-frame halo gives
    # the same labels as the whole clip (the multi-GPU sharding rule)
    f0 = 333_333
    seg = audio[160 * f0: 160 * (f0 + 100_000) + 240 + 160 * 5 + 1].contiguous()
    lab_seg = pipe.labels(seg)
    assert torch.equal(lab_seg[:100_000], lab1[f0: f0 + 100_000])
    # the MFCC of a clip equals the MFCC of its explicit frame matrix
    m = pipe.mfcc(audio[: 160 * 999 + 401].contiguous())
    fm = audio[: 160 * 999 + 400].unfold(0, 400, 160).contiguous()
    m2 = pipe.plan.mfcc(fm)
    assert torch.equal(m, m2)
    # labels of silent windows are class 0 (NaN features)
    c = 5_000_000 // 160 + 10
    assert int(lab1[c - 2]) == 0


@pytest.mark.parametrize("nf", [26, 40])
def test_compiled_tables_match_runtime_path(torch_cuda, golden, nf):
    """The compile-time Mel26/Mel40 kernels and the runtime-table kernel agree."""
    from vad_amd.plan import MfccPlan
    fb = O.get_mel_filterbanks(300, 8000, 512, nf, 16000)
    p = MfccPlan(fb)
    assert p.variant == (1 if nf == 26 else 2)
    clip = torch_cuda.from_numpy(O.synth_clip(160 * 2000 + 401, seed=9)).cuda()
    m_spec = p.clip_mfcc(clip).cpu().numpy()
    p.set_variant(0)
    assert p.variant == 0
    m_gen = p.clip_mfcc(clip).cpu().numpy()
    assert frame_rel(m_spec, m_gen).max() <= 1e-5
    ref = O.mfcc_batch(clip.cpu().numpy(), fb)
    assert_mfcc_close(m_spec, ref)
    assert_mfcc_close(m_gen, ref)
    # a non-reference bank stays on the runtime path
    assert MfccPlan(O.get_mel_filterbanks(100, 4000, 512, 32, 16000)).variant == 0


# ---------------------------------------------------------------------------
# decision tree (decision_classifier_trainer.py:26-35, the classifier vad.py
# deploys) -- sklearn's traversal on the GPU node table
# ---------------------------------------------------------------------------
def _tree(golden):
    from vad_amd.tree import TreeClassifier
    g = golden("tree")
    return g, TreeClassifier(g["feature"], g["threshold"], g["left"], g["right"], g["leaf"],
                             g["nan_left"], g["classes"], int(g["n_features"]))


def test_tree_predict_matches_sklearn(torch_cuda, golden):
    g, t = _tree(golden)
    assert np.array_equal(t.predict(g["x_test"]), g["y_test"])


def test_tree_window_labels_on_clip(torch_cuda, golden):
    """Fused window features + tree walk == the oracle walk over the GPU's own
    fp32 features (so the comparison is exact), analyser and offline modes;
    plus VadPipeline(labels) with the tree."""
    from vad_amd import _lib
    from vad_amd.pipeline import VadPipeline
    from vad_amd.plan import window_features
    g, t = _tree(golden)
    tree = {k: g[k] for k in ("feature", "threshold", "left", "right", "leaf", "nan_left",
                              "classes")} | {"n_features": int(g["n_features"])}
    clip = O.synth_clip(O.samples_for_frames(3000), 41)
    clip[160 * 1000:160 * 1100] = 0.0  # digital silence: NaN features
    pipe = VadPipeline(ffn=t)
    a = torch_cuda.from_numpy(clip).cuda()
    m = pipe.mfcc(a)
    for mode in (_lib.FEAT_ANALYSER, _lib.FEAT_OFFLINE):
        feats = window_features(m, mode).cpu().numpy()
        ref = O.tree_predict(tree, feats)
        got = g["classes"][t.window_labels(m, mode).cpu().numpy()]
        assert np.array_equal(got, ref)
    assert np.isnan(window_features(m, _lib.FEAT_ANALYSER).cpu().numpy()).any()
    lab = pipe.labels(a).cpu().numpy()
    assert np.array_equal(g["classes"][lab], O.tree_predict(tree, window_features(m).cpu().numpy()))


def test_tree_window_threshold_ties(torch_cuda, golden):
    """The LDS walk compares float features with thresholds rounded down to
    float; sklearn compares in double.  Thresholds set exactly to feature
    values the windows produce, and one double ulp above / below them, must
    give the oracle's (double-comparison) labels."""
    from vad_amd.plan import window_features
    from vad_amd.tree import TreeClassifier
    g, _ = _tree(golden)
    clip = O.synth_clip(O.samples_for_frames(2000), 43)
    from vad_amd.pipeline import VadPipeline
    m = VadPipeline().mfcc(torch_cuda.from_numpy(clip).cuda())
    feats = window_features(m).cpu().numpy()
    rng = np.random.default_rng(5)
    thr = g["threshold"].copy()
    inner = np.nonzero(g["feature"] >= 0)[0]
    for k, i in enumerate(inner):  # each internal node: a feature value seen at that node's feature
        col = feats[:, g["feature"][i]]
        v = float(col[rng.integers(len(col))])
        if not np.isfinite(v):
            continue
        thr[i] = (v, np.nextafter(v, np.inf), np.nextafter(v, -np.inf))[k % 3]
    tree = {"feature": g["feature"], "threshold": thr, "left": g["left"], "right": g["right"],
            "leaf": g["leaf"], "nan_left": g["nan_left"], "classes": g["classes"],
            "n_features": int(g["n_features"])}
    t = TreeClassifier(g["feature"], thr, g["left"], g["right"], g["leaf"], g["nan_left"],
                       g["classes"], int(g["n_features"]))
    got = g["classes"][t.window_labels(m).cpu().numpy()]
    assert np.array_equal(got, O.tree_predict(tree, feats))
    assert np.array_equal(t.predict(feats), O.tree_predict(tree, feats))  # the global row walk


class _HostTree:
    """The same sklearn tree kept on the host (the reference's call path)."""

    def __init__(self, clf):
        self.clf = clf

    def predict(self, x):
        return self.clf.predict(x)


def test_analyser_with_pickled_sklearn_tree(torch_cuda, golden, tmp_path):
    """SKLearnAnalyzer(pickled DecisionTreeClassifier): the tree moves to the
    GPU and the feed_frame trace equals the host-sklearn call path."""
    from sklearn.tree import DecisionTreeClassifier
    from vad_amd.sklearn_analyser import SKLearnAnalyzer
    from vad_amd.tree import TreeClassifier
    ga = golden("analyser")
    gt = golden("tree")
    clf = DecisionTreeClassifier(min_samples_split=22, max_depth=25, min_samples_leaf=20,
                                 random_state=0).fit(np.nan_to_num(gt["x_test"]), gt["y_test"])
    p1 = tmp_path / "tree.cls"
    with open(p1, "wb") as f:
        pickle.dump(clf, f)
    p2 = tmp_path / "host.cls"
    with open(p2, "wb") as f:
        pickle.dump(_HostTree(clf), f)
    an_gpu = SKLearnAnalyzer(str(p1))
    assert isinstance(an_gpu.classifier, TreeClassifier)
    an_host = SKLearnAnalyzer(str(p2))
    for an in (an_gpu, an_host):
        an.load_init_inactive_frames(list(ga["noise"]))
    stream = list(ga["stream"])
    for fr in stream:
        r1, r2 = an_gpu.feed_frame(fr), an_host.feed_frame(fr)
        assert (r1 is None and r2 is None) or (r1 is r2)


# ---------------------------------------------------------------------------
# fft_n other than 512 (mfcc.py:59-61 takes any length; every reference call
# site passes 512): the direct-DFT path, against the oracle's pocketfft
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("fft_n,n_filters", [(256, 16), (400, 26), (401, 26), (1024, 26), (2048, 40),
                                              (8192, 26)])
def test_other_fft_lengths(torch_cuda, fft_n, n_filters):
    torch = torch_cuda
    from vad_amd import mfcc as M
    from vad_amd.plan import MfccPlan
    rng = np.random.default_rng(fft_n)
    fb = O.get_mel_filterbanks(300, 8000, fft_n, n_filters, 16000)
    assert np.isfinite(fb).all()
    for L in (400, 300, fft_n + 100):  # zero-padded and truncated frames
        frame = np.round(rng.standard_normal(L) * 3000).astype(np.float32)
        s = M.get_spec_mag(frame, fft_n)
        ref = O.get_spec_mag(frame, fft_n)
        assert s.dtype == np.float32 and s.shape == ref.shape == (fft_n // 2,)
        assert frame_rel(s, ref) <= SPEC_TOL
        assert_mfcc_close(M.get_mfcc(frame, fft_n, fb, 13)[None], O.get_mfcc(frame, fft_n, fb, 13)[None])
        assert_mfcc_close(M.get_mfcc_from_spec(ref, fb, 13)[None], O.get_mfcc_from_spec(ref, fb, 13)[None])
    # a clip through a plan: every frame, fp32 and int16 PCM (identical)
    clip = O.synth_clip(O.samples_for_frames(300), seed=fft_n)
    p = MfccPlan(fb, 13, fft_n)
    assert p.variant == 0
    a = torch.from_numpy(clip).cuda()
    got = p.clip_mfcc(a).cpu().numpy()
    assert_mfcc_close(got, O.mfcc_batch(clip, fb, fft_n=fft_n))
    assert np.array_equal(p.clip_mfcc(a.to(torch.int16)).cpu().numpy(), got)


def test_other_fft_length_pipeline(torch_cuda):
    """A 1024-point MFCC config through VadPipeline (workspace form) and the
    three-kernel streaming step; the fused kernel and the hop kernel are the
    fft_n = 512 pipeline and say so."""
    torch = torch_cuda
    from vad_amd import _lib
    from vad_amd.config import MfccConfig
    from vad_amd.ffn import TOPOLOGY_BL13, FFNClassifier, random_layers
    from vad_amd.pipeline import VadPipeline
    from vad_amd.stream import StreamBatch
    layers = random_layers(TOPOLOGY_BL13, seed=9)
    pipe = VadPipeline(FFNClassifier(layers), cfg=MfccConfig(fft_n=1024))
    clip = O.synth_clip(O.samples_for_frames(3000), seed=91)
    lab = pipe.labels(torch.from_numpy(clip).cuda()).cpu().numpy()
    fb = O.get_mel_filterbanks(300, 8000, 1024, 26, 16000)
    x = O.analyser_features_fast(O.mfcc_batch(clip, fb, fft_n=1024))[:, :13]
    sure = O.ffn_margin(x, layers) > MARGIN_TOL
    np.testing.assert_array_equal(lab[sure], O.ffn_labels(x, layers)[sure])
    assert not pipe.fusable
    with pytest.raises(RuntimeError):  # VadError: VAD_EUNSUPPORTED
        pipe.labels(torch.from_numpy(clip).cuda(), fused=True)
    # the three-kernel streaming step runs the same path; 3 identical streams
    sb = StreamBatch(3, FFNClassifier(layers), cfg=MfccConfig(fft_n=1024), kernel="three")
    sb.prime(torch.from_numpy(np.stack([clip[:240]] * 3)).cuda())
    outs = [sb.step(torch.from_numpy(np.stack([clip[240 + 160 * t: 400 + 160 * t]] * 3)).cuda())
            .cpu().numpy().copy() for t in range(12)]
    for t in range(5, 12):
        if sure[t - 5]:
            assert outs[t].tolist() == [lab[t - 5]] * 3
    hop = StreamBatch(3, FFNClassifier(layers), cfg=MfccConfig(fft_n=1024), kernel="hop")
    hop.prime(torch.from_numpy(np.stack([clip[:240]] * 3)).cuda())
    with pytest.raises(RuntimeError):
        hop.step(torch.from_numpy(np.stack([clip[240:400]] * 3)).cuda())


@pytest.mark.parametrize("mfcc_n", [1, 12, 16])
def test_other_coefficient_counts(torch_cuda, mfcc_n):
    """get_mfcc's mfcc_n (mfcc.py:67-78; the analyser's mfcc_num) other than
    13, up to VAD_MAX_MFCC: the runtime-table kernel's lifter x DCT rows,
    the analyser window features (3 mfcc_n columns) and a generic-topology
    FFN on them, the clip path and the one-kernel hop, vs the oracle."""
    import torch
    from vad_amd.config import MfccConfig
    from vad_amd.ffn import FFNClassifier, random_layers
    from vad_amd.pipeline import VadPipeline
    from vad_amd.plan import window_features
    from vad_amd.stream import StreamBatch
    cfg = MfccConfig(n_mfcc=mfcc_n)
    F = 3000
    clip = O.synth_clip(O.samples_for_frames(F), seed=41)
    fb = O.get_mel_filterbanks(300, 8000, 512, 26, 16000)
    ref = O.mfcc_batch(clip, fb, mfcc_n=mfcc_n)
    layers = random_layers((3 * mfcc_n, 32, 2), seed=9)
    pipe = VadPipeline(FFNClassifier(layers), cfg=cfg)
    a = torch.from_numpy(clip).cuda()
    m = pipe.mfcc(a)
    got = m.cpu().numpy().astype(np.float64)
    assert got.shape == ref.shape == (F, mfcc_n)
    # norm-wise per frame against the frame's 13-coefficient
    # norm at least: with one coefficient, c0 alone can sit near 0
    ref13 = O.mfcc_batch(clip, fb)
    den = np.maximum(np.linalg.norm(ref, axis=1), np.linalg.norm(ref13, axis=1))
    rel = np.linalg.norm(got - ref, axis=1) / den
    assert rel.max() <= 1e-4, rel.max()
    x = O.analyser_features_fast(ref)
    feats = window_features(m).cpu().numpy()
    assert feats.shape == x.shape == (F - 5, 3 * mfcc_n)
    labels = pipe.labels(a).cpu().numpy()
    sure = O.ffn_margin(x, layers) > MARGIN_TOL
    np.testing.assert_array_equal(labels[sure], O.ffn_labels(x, layers)[sure])
    # the streaming hop on the same frames: its window labels agree where decisive
    T = 64
    sb = StreamBatch(2, FFNClassifier(layers), cfg=cfg, kernel="hop")
    sb.prime(torch.from_numpy(np.stack([clip[:240]] * 2)).cuda())
    hl = np.stack([sb.step(torch.from_numpy(np.stack([clip[240 + 160 * t: 400 + 160 * t]] * 2)).cuda())
                   .cpu().numpy().copy() for t in range(T)])
    assert (hl[:5] == 255).all()
    ok = sure[:T - 5]
    np.testing.assert_array_equal(hl[5:, 0][ok], O.ffn_labels(x, layers)[:T - 5][ok])
    np.testing.assert_array_equal(hl[:, 0], hl[:, 1])


def test_other_sample_rate(torch_cuda):
    """An 8 kHz configuration (get_mel_filterbanks' sample_rate, mfcc.py:39-56;
    the analyser's sample_rate): 20 ms frames, 10 ms hop, 256-point FFT,
    26 filters up to 4 kHz -- the runtime-table / generic-FFT path, MFCCs
    vs the oracle norm-wise per frame."""
    import torch
    from vad_amd.config import MfccConfig
    from vad_amd.pipeline import VadPipeline
    cfg = MfccConfig(sample_rate=8000, frame_size=160, hop=80, fft_n=256, low_hz=300, high_hz=4000)
    F = 2000
    clip = O.synth_clip(80 * (F - 1) + 161, seed=43)
    fb = O.get_mel_filterbanks(300, 4000, 256, 26, 8000)
    ref = O.mfcc_batch(clip, fb, frame_size=160, step=80, fft_n=256)
    got = VadPipeline(cfg=cfg).mfcc(torch.from_numpy(clip).cuda()).cpu().numpy().astype(np.float64)
    assert got.shape == ref.shape == (F, 13)
    rel = np.linalg.norm(got - ref, axis=1) / np.linalg.norm(ref, axis=1)
    assert rel.max() <= 1e-4, rel.max()


def test_nonfinite_samples(torch_cuda):
    """Corrupted audio: a NaN and an inf sample.  The reference's float path
    (mfcc.py:59-78) turns every frame that contains one into a NaN MFCC row
    (np.fft spreads it over every bin) and its windows into NaN feature rows,
    which the Keras forward keeps NaN and np.argmax maps to class 0; frames
    without one are untouched.  The device gives the same NaN rows, finite
    rows within the usual tolerance elsewhere, and class 0 on every window
    that sees a NaN row -- in the two-kernel clip form, the fused kernel and
    the one-kernel streaming hop."""
    import torch
    from vad_amd.ffn import FFNClassifier, random_layers
    from vad_amd.pipeline import VadPipeline
    F = 400
    clip = O.synth_clip(O.samples_for_frames(F), seed=47).astype(np.float32)
    clip[160 * 100 + 7] = np.nan
    clip[160 * 300 + 200] = np.inf
    fb = O.get_mel_filterbanks(300, 8000, 512, 26, 16000)
    with np.errstate(invalid="ignore", over="ignore"):
        ref = O.mfcc_batch(clip, fb)
    layers = random_layers((13, 64, 64, 2), seed=3)
    pipe = VadPipeline(FFNClassifier(layers))
    a = torch.from_numpy(clip).cuda()
    got = pipe.mfcc(a).cpu().numpy().astype(np.float64)
    bad_ref = ~np.isfinite(ref).all(axis=1)
    bad_got = ~np.isfinite(got).all(axis=1)
    assert bad_ref.any()
    np.testing.assert_array_equal(bad_got, bad_ref)
    ok = ~bad_ref
    rel = np.linalg.norm(got[ok] - ref[ok], axis=1) / np.linalg.norm(ref[ok], axis=1)
    assert rel.max() <= 1e-4
    labels = pipe.labels(a).cpu().numpy()
    win_bad = np.array([bad_ref[i:i + 5].any() for i in range(F - 5)])
    assert (labels[win_bad] == 0).all()
    # the fused kernel and the one-kernel streaming hop on the same samples
    np.testing.assert_array_equal(pipe.labels(a, fused=True).cpu().numpy(), labels)
    from vad_amd.stream import StreamBatch
    sb = StreamBatch(1, FFNClassifier(layers), kernel="hop")
    sb.prime(a[:240].reshape(1, 240))
    hl = np.array([int(sb.step(a[240 + 160 * t: 400 + 160 * t].reshape(1, 160).contiguous())[0])
                   for t in range(F)])
    assert (hl[:5] == 255).all()
    assert (hl[5:][win_bad] == 0).all()
    with np.errstate(invalid="ignore"):
        x = O.analyser_features_fast(ref)[:, :13]
        sure = O.ffn_margin(x, layers) > MARGIN_TOL
    np.testing.assert_array_equal(labels[sure & ~win_bad], O.ffn_labels(x, layers)[sure & ~win_bad])


@pytest.mark.gpu
def test_feature_range_edges(torch_cuda):
    """The analyser normalisation is fp32 with v_rsq_f32 on 0.2 var 2^24
    (features.h): caller-supplied MFCC rows whose 5-frame std lies in
    [2^-60, 2^50] give the oracle's Mn (and deltas) to fp32 rounding; past
    that the documented edges hold (include/vad_amd.h, vad_features_f32):
    std ~2^56 overflows the scaled variance -> Mn = 0, std ~2^-90 underflows
    the squares -> Mn = +-inf.  Log-MFCCs of any audio sit far inside."""
    torch = torch_cuda
    from vad_amd.plan import window_features
    rng = np.random.default_rng(7)
    base = rng.standard_normal((64, 13)).astype(np.float32)
    for k in (-60, -30, 0, 20, 50):
        m = (base * np.float32(2.0 ** k)).astype(np.float32)
        got = window_features(torch.from_numpy(m).cuda()).cpu().numpy().astype(np.float64)
        ref = O.analyser_features_fast(m)
        assert np.isfinite(got).all(), k
        np.testing.assert_allclose(got[:, :13], ref[:, :13], rtol=1e-5, atol=1e-5, err_msg=f"Mn at 2^{k}")
        scale = 2.0 ** k
        np.testing.assert_allclose(got[:, 13:26] / scale, ref[:, 13:26] / scale, rtol=0, atol=1e-5,
                                   err_msg=f"M+1 - M-1 at 2^{k}")
        # (M+2 - Mn) - (Mn - M-2) mixes the O(1) Mn with rows at the scale
        np.testing.assert_allclose(got[:, 26:], ref[:, 26:], rtol=1e-5, atol=1e-5 * max(1.0, scale),
                                   err_msg=f"second deltas at 2^{k}")
    hi = (base * np.float32(2.0 ** 56)).astype(np.float32)
    got = window_features(torch.from_numpy(hi).cuda()).cpu().numpy()
    assert (got[:, :13] == 0).all()  # scaled variance overflows: rsq(inf) = 0
    assert np.isfinite(got[:, 13:26]).all()  # M+1 - M-1 unaffected
    lo = (base * np.float32(2.0 ** -90)).astype(np.float32)
    got = window_features(torch.from_numpy(lo).cuda()).cpu().numpy()
    assert np.isinf(got[:, :13]).all()  # squares underflow: var 0, e2 / 0


def test_plan_destroy_waits_for_pending_work(torch_cuda):
    """A plan collected while its kernels are still queued (the Python object
    dropped right after an asynchronous launch on a side stream): destroy
    frees the plan's device tables with hipFree, which waits for the device,
    so the queued launches still read live tables -- labels and MFCCs equal
    a run whose plans stay alive."""
    import gc
    import torch
    from vad_amd.ffn import TOPOLOGY_BL13, FFNClassifier, random_layers
    from vad_amd.plan import MfccPlan
    F = 400_000
    clip = torch.from_numpy(O.synth_clip(O.samples_for_frames(F), seed=41)).cuda()
    fb = O.get_mel_filterbanks(300, 8000, 512, 26, 16000)
    lay = random_layers(TOPOLOGY_BL13, seed=3)
    keep_p, keep_c = MfccPlan(fb), FFNClassifier(lay)
    m_ref = keep_p.clip_mfcc(clip)
    lab_ref = keep_c.plan.window_labels(m_ref)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        m = torch.empty_like(m_ref)
        lab = torch.empty_like(lab_ref)
        for _ in range(3):  # a queue of work behind the launches that use the plans
            MfccPlan(fb).clip_mfcc(clip, out=m, stream=side)
            FFNClassifier(lay).plan.window_labels(m, out=lab, stream=side)
            gc.collect()  # the plans above are unreferenced now
    side.synchronize()
    assert torch.equal(m, m_ref) and torch.equal(lab, lab_ref)
