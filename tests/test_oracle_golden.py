"""Pin the CPU oracle (oracle/vad_oracle.py) against the golden vectors that
tests/golden/gen_golden.py produced by running the unmodified reference."""
import numpy as np
import pytest

from oracle import vad_oracle as O


def frame_rel(a, b):
    """Per-frame L2-relative error (SURVEY.md 8(c) tolerance definition)."""
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return np.linalg.norm(a - b, axis=-1) / np.maximum(np.linalg.norm(b, axis=-1), 1e-300)


@pytest.mark.parametrize("name", ["fb_26", "fb_40", "fb_20_0_8000", "fb_32_100_4000"])
def test_filterbanks(golden, name):
    g = golden("filterbanks")
    lo, hi, nf, sr = g[name + "_params"]
    fb = O.get_mel_filterbanks(lo, hi, 512, int(nf), sr)
    np.testing.assert_array_equal(fb, g[name])
    hz = O.hz_from_mel(O.mel_from_hz(lo, hi, int(nf)))
    np.testing.assert_array_equal(O.convert_to_fft_bins(sr, hz, 512), g[name + "_bins"])


def test_fb26_structure(golden):
    fb = golden("filterbanks")["fb_26"]
    assert (fb != 0).sum() == 444
    assert ((fb != 0).sum(axis=0) <= 2).all()  # each bin feeds at most two filters


def test_spec_mag_exact(golden):
    g = golden("frames")
    spec = O.spec_batch(g["frames"])
    np.testing.assert_array_equal(spec, g["spec"])  # same pocketfft float32 path
    for i, f in enumerate(g["frames"][:8]):
        np.testing.assert_array_equal(O.get_spec_mag(f), g["spec"][i])


@pytest.mark.parametrize("nf,key", [(26, "mfcc26"), (40, "mfcc40")])
def test_mfcc_from_spec(golden, nf, key):
    g = golden("frames")
    fb = O.get_mel_filterbanks(300, 8000, 512, nf, 16000)
    m = O.get_mfcc_from_spec(g["spec"], fb, 13)
    ref = g[key]
    # fp64 restatement of scipy's DCT: per-frame agreement far inside 1e-4
    assert frame_rel(m, ref).max() < 1e-12
    # digital silence: c0 = log10(eps)*sqrt(n_filters)
    assert abs(ref[0, 0] - np.log10(np.finfo(float).eps) * np.sqrt(nf)) < 1e-9


@pytest.mark.parametrize("L", [800, 512, 256, 401])
def test_other_frame_lengths(golden, L):
    g = golden("frames")
    fb = O.get_mel_filterbanks(300, 8000, 512, 26, 16000)
    fr = g[f"frames_{L}"]
    np.testing.assert_array_equal(O.spec_batch(fr), g[f"spec_{L}"])
    m = np.stack([O.get_mfcc(f, 512, fb, 13) for f in fr])
    assert frame_rel(m, g[f"mfcc26_{L}"]).max() < 1e-12


def test_framing_counts(golden):
    g = golden("clip")
    for L, c in zip(g["lens"], g["counts"]):
        assert O.n_frames(int(L)) == c
        assert len(O.split_into_frames(np.zeros(int(L)))) == c
        assert len(O.frame_matrix(np.zeros(int(L), np.float32))) == c


def test_offline_features(golden):
    g = golden("clip")
    fb = O.get_mel_filterbanks(300, 8000, 512, 26, 16000)
    m = O.mfcc_batch(g["clip"], fb)
    assert frame_rel(m, g["mfcc"]).max() < 1e-12
    f = O.offline_features(m)
    ref = g["features"]
    assert f.shape == ref.shape == (93, 3, 13)
    assert frame_rel(f.reshape(len(f), -1), ref.reshape(len(ref), -1)).max() < 1e-12


def _layers(w, prefix, n, b_last=None):
    lay = [(w[f"{prefix}_W{i}"], w[f"{prefix}_b{i}"]) for i in range(n)]
    if b_last is not None:
        lay[-1] = (lay[-1][0], b_last)
    return lay


def test_analyser_trace(golden):
    g = golden("analyser")
    w = golden("ffn")
    lay = _layers(w, "ref39", 4)
    an = O.AnalyserOracle(O.FFNPredictor(lay))
    an.load_init_inactive_frames(list(g["noise"]))
    stream = list(g["stream"])
    rets, feats = [], []
    for f in stream:
        if len(an.frames_buffer) == 5:
            feats.append(an.features())
        r = an.feed_frame(f)
        rets.append(-1 if r is None else next(i for i, s in enumerate(stream) if s is r))
    np.testing.assert_array_equal(rets, g["returns"])
    fx = np.asarray(feats)
    ref = g["features"]
    # Constant (digital-silence) windows: std = 0 -> 0/0 = NaN.  Which of the
    # 13 coefficients come out NaN depends on the last-ulp noise of each DCT
    # implementation (c1..c12 of a constant log-energy vector are ~1e-14), but
    # every such row holds a NaN, so its label is 0 either way.
    nan_rows = np.isnan(ref).any(axis=1)
    np.testing.assert_array_equal(np.isnan(fx).any(axis=1), nan_rows)
    assert nan_rows.sum() >= 5
    assert np.allclose(fx[~nan_rows], ref[~nan_rows], rtol=1e-9, atol=1e-9)


def test_analyser_errors(golden):
    g = golden("analyser")
    w = golden("ffn")
    assert str(g["error_noinit"]) == "0:TypeError"
    assert str(g["error_badinit"]) == "ValueError"
    an = O.AnalyserOracle(O.FFNPredictor(_layers(w, "ref39", 4)))
    with pytest.raises(TypeError):
        an.feed_frame(g["stream"][0])
    with pytest.raises(ValueError):
        an.load_init_inactive_frames(list(g["noise"][:4]))
    an = O.AnalyserOracle(O.FFNPredictor(_layers(w, "ref39", 4, w["ref39_b3_music"])))
    an.load_init_inactive_frames(list(g["noise"]))
    k = int(str(g["error_music"]).split(":")[0])
    for f in g["stream"][:k]:
        an.feed_frame(f)
    with pytest.raises(AssertionError):
        an.feed_frame(g["stream"][k])


def test_ffn_labels(golden):
    w = golden("ffn")
    x = w["test_x"]
    np.testing.assert_array_equal(O.ffn_labels(x, _layers(w, "ref39", 4)), w["test_labels_ref39"])
    np.testing.assert_array_equal(O.ffn_labels(x[:, :13], _layers(w, "bl13", 3)),
                                  w["test_labels_bl13"])
    # the fixture features are the analyser features of the fixture clip
    fb = O.get_mel_filterbanks(300, 8000, 512, 26, 16000)
    fx = O.analyser_features(O.mfcc_batch(w["test_clip"], fb))
    np.testing.assert_array_equal(np.isnan(fx).any(axis=1), np.isnan(x).any(axis=1))


def test_nan_label_is_zero():
    lay = [(np.ones((39, 4), np.float32), np.zeros(4, np.float32)),
           (np.ones((4, 3), np.float32), np.array([0, 5, 1], np.float32))]
    x = np.ones((2, 39))
    x[0, 5] = np.nan
    assert list(O.ffn_labels(x, lay)) == [0, 1]


def test_fast_analyser_features_equal_loop(golden):
    w = golden("ffn")
    fb = O.get_mel_filterbanks(300, 8000, 512, 26, 16000)
    m = O.mfcc_batch(w["test_clip"], fb)
    a = O.analyser_features(m)
    b = O.analyser_features_fast(m)
    np.testing.assert_array_equal(np.isnan(a), np.isnan(b))
    ok = ~np.isnan(a)
    assert np.allclose(a[ok], b[ok], rtol=1e-12, atol=1e-12)


# ---------------------------------------------------------------------------
# decision tree (decision_classifier_trainer.py:26-35)
# ---------------------------------------------------------------------------
def _tree_from_fixture(g):
    return {k: g[k] for k in ("feature", "threshold", "left", "right", "leaf", "nan_left",
                              "classes")} | {"n_features": int(g["n_features"])}


def test_tree_oracle_matches_sklearn_fixture(golden):
    """The restated traversal reproduces the predictions sklearn recorded
    (fixture made by tests/golden/gen_tree.py, incl. NaN feature rows)."""
    g = golden("tree")
    pred = O.tree_predict(_tree_from_fixture(g), g["x_test"])
    assert np.array_equal(pred, g["y_test"])
    assert np.isnan(g["x_test"]).any()


def test_tree_oracle_matches_live_sklearn():
    """Pin the restatement against the installed sklearn on fresh data: ties
    at thresholds (float32 grid), NaNs, three classes."""
    from sklearn.tree import DecisionTreeClassifier
    rng = np.random.default_rng(3)
    X = np.round(rng.standard_normal((3000, 7)) * 4).astype(np.float32) / 4  # many exact ties
    y = (X[:, 0] + X[:, 1] > 0).astype(int) + (X[:, 2] > 1).astype(int)
    X[rng.random(X.shape) < 0.02] = np.nan
    clf = DecisionTreeClassifier(min_samples_split=22, max_depth=25, min_samples_leaf=20,
                                 random_state=1).fit(X, y)
    Xt = np.round(rng.standard_normal((2000, 7)) * 4).astype(np.float32) / 4
    Xt[rng.random(Xt.shape) < 0.05] = np.nan
    assert np.array_equal(O.tree_predict(O.tree_arrays(clf), Xt), clf.predict(Xt))


def _sklearn_mlp(layers, n_classes):
    """scikit-learn's MLPClassifier carrying `layers` (Keras (in, out) layout,
    relu hidden layers): an independent implementation of the forward the
    oracle restates (ffn_trainer.py:106-116).  Two classes: sklearn's binary
    output is one logistic unit, i.e. the softmax of (z0, z1) folded into
    z1 - z0."""
    import warnings
    from sklearn.exceptions import ConvergenceWarning
    from sklearn.neural_network import MLPClassifier
    hidden = tuple(w.shape[1] for w, _ in layers[:-1])
    clf = MLPClassifier(hidden_layer_sizes=hidden, activation="relu", max_iter=1, random_state=0)
    rng = np.random.default_rng(0)
    xs = rng.standard_normal((4 * n_classes, layers[0][0].shape[0]))
    with warnings.catch_warnings():
        warnings.simplefilter("ignore", ConvergenceWarning)
        clf.fit(xs, np.arange(4 * n_classes) % n_classes)
    ws = [np.asarray(w, np.float64) for w, _ in layers]
    bs = [np.asarray(b, np.float64) for _, b in layers]
    if n_classes == 2:
        ws[-1] = (ws[-1][:, 1] - ws[-1][:, 0])[:, None]
        bs[-1] = np.array([bs[-1][1] - bs[-1][0]])
    clf.coefs_, clf.intercepts_ = ws, bs
    return clf


@pytest.mark.parametrize("topo,n_classes", [("ref39", 3), ("bl13", 2)])
def test_ffn_oracle_matches_sklearn_mlp(golden, topo, n_classes):
    """The fp64 FFN restatement (Keras is absent) against live
    scikit-learn's MLP forward on the fixture weights and feature rows:
    probabilities to 1e-12 and labels exactly (finite rows: sklearn rejects
    NaN input; the NaN rule is test_nan_label_is_zero's)."""
    g = golden("ffn")
    n = 4 if topo == "ref39" else 3
    layers = [(g[f"{topo}_W{i}"], g[f"{topo}_b{i}"]) for i in range(n)]
    x = g["test_x"] if topo == "ref39" else g["test_x"][:, :13]
    x = x[np.isfinite(x).all(axis=1)]
    assert len(x) > 500
    clf = _sklearn_mlp(layers, n_classes)
    _, p = O.ffn_forward(x, layers)
    sp = clf.predict_proba(x)
    np.testing.assert_allclose(sp, p, rtol=0, atol=1e-12)
    np.testing.assert_array_equal(clf.predict(x), O.ffn_labels(x, layers))


def _cyclotomic_degree(taps, fft_n):
    """Least degree of a nonzero rational polynomial vanishing at w^k for
    every k in taps (w = exp(-2 pi i / fft_n), fft_n a power of two): the sum
    of phi(m) over the distinct orders m = fft_n / gcd(k, fft_n) -- X[k] = 0
    for a frame with rational samples x iff Phi_m divides sum x[n] z^n, and
    distinct cyclotomic polynomials are coprime."""
    from math import gcd
    orders = {fft_n // gcd(int(k), fft_n) for k in taps}
    return sum(1 if m == 1 else m // 2 for m in orders)


def test_spectral_null_reachability():
    """Which mel filters can lie wholly on exact spectral nulls (energy
    exactly 0 -> eps in exact arithmetic, rounding noise in an FFT that does
    not cancel exactly) for a reference-configuration frame: 400 samples
    zero-padded to 512, so sum x[n] z^n has degree <= 399.  26 filters: none
    (the least degree is 400, filter 1, bins 13..17).  40 filters: filter 9
    alone (bins 30..33: Phi_256 Phi_512 Phi_16, degree 392), and the
    fixture's (z^256+1)(z^128+1)(z^8+1) frames null it exactly -- checked in
    exact cyclotomic arithmetic (gen_nulls.exact_null_bins), not by FFT."""
    import sys, os
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
    from gen_nulls import comb_frames, exact_null_bins
    deg = {}
    for nf in (26, 40):
        fb = O.get_mel_filterbanks(300, 8000, 512, nf, 16000)
        deg[nf] = [_cyclotomic_degree(np.flatnonzero(fb[m]), 512) for m in range(nf)]
    assert min(deg[26]) == 400 and deg[26].index(400) == 1
    assert [m for m in range(40) if deg[40][m] <= 399] == [9] and deg[40][9] == 392
    fb40 = O.get_mel_filterbanks(300, 8000, 512, 40, 16000)
    taps9 = np.flatnonzero(fb40[9])
    hit = [i for i, f in enumerate(comb_frames()) if exact_null_bins(f)[taps9].all()]
    assert len(hit) >= 3
    # the deep-fuzz configuration (fft_n 300 is not a power of two: Phi_m of
    # other orders; the reachability there is what test_gpu_fuzz excludes)


def test_null_fixture_pins_oracle(golden):
    """The oracle on the spectral-null fixture (tests/golden/nulls.npz, the
    reference's own outputs): spectra bit-exact (pocketfft), exact zeros on
    every exact null bin, MFCCs within 1e-6 at 26 and 40 filters."""
    g = golden("nulls")
    spec = O.spec_batch(g["frames"], 512)
    np.testing.assert_array_equal(spec, g["spec"])
    np.testing.assert_array_equal(spec[g["null_bins"]], 0.0)
    for nf in (26, 40):
        fb = O.get_mel_filterbanks(300, 8000, 512, nf, 16000)
        m = np.stack([O.get_mfcc_from_spec(s, fb, 13) for s in spec])
        np.testing.assert_allclose(m, g[f"mfcc{nf}"], rtol=1e-6, atol=1e-6)
