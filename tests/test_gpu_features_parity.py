"""The analyser's feature rows, value for value, against the reference run.

SKLearnAnalyzer.feed_frame builds [Mn, D1, D2] with Mn = (M_c - mean5) / std5
(realtime_analysis/sklearn_analyser.py:52-71, 103-107) and hands the (1, 39)
float64 row to classifier.predict.  tests/golden/analyser.npz holds the rows
the UNMODIFIED reference passed to predict (gen_golden.py's recorder), for the
198-frame stream and for vad.py's 800-value blocks.  Here the drop-in analyser
replays the same calls with a recording classifier and every recorded row is
compared with the reference's row:

  NaN positions  identical (a digital-silence window is 0/0 in Mn and D2);
  values         |d| <= bound elementwise, the first-order propagation of the
                 device MFCC error through the window statistics:
                   E    = U_MFCC * max_d ||M_d||   (per-frame MFCC error bound)
                   Mn   : ELEM_C * 2 E (1 + |Mn|) / std     (std in the divisor:
                          an almost-flat coefficient amplifies any MFCC rounding)
                   D1   : ELEM_C * 2 E
                   D2   : ELEM_C * (2 E + 2 * bound(Mn))
                 U_MFCC = 1e-6 covers the device MFCC error (4.8e-7 worst
                 frame in smoke / the C3 test) and the fp32 window statistics
                 (2^-24 |M| per operation);
  rows           ||d||_2 / ||ref||_2 <= ROW_TOL on every fixture row (a
                 host simulation of 3e-7 MFCC noise gives 1.2e-5 worst).

The same bound holds on a C3-size clip (1M frames) against the oracle's
features of the oracle's fp64 MFCCs, where ill-conditioned windows exist (a
coefficient whose 5-frame std is ~1e-5 of the frame norm): there the per-row
1e-4 holds for >= 99.5 % of rows and the elementwise bound for all.

Finally the GPU decision-tree analyser's returns on the fixture stream equal
the returns the tree gives on the REFERENCE rows (O.tree_predict, sklearn's
double comparison), except on rows whose decision path passes within the
feature bound of a threshold (counted; none on this fixture).
"""
import pickle

import numpy as np
import pytest

from oracle import vad_oracle as O

pytestmark = pytest.mark.gpu

U_MFCC = 1e-6
ELEM_C = 8.0
ROW_TOL = 1e-4


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    return torch


class FeatureRecorder:
    """A foreign classifier: records every row the analyser passes to predict."""

    def __init__(self, labels):
        self.labels = list(labels)
        self.rows = []

    def predict(self, x):
        self.rows.append(np.array(x))
        return np.array([self.labels[len(self.rows) - 1]])


def windows(mfcc):
    """(R, 5, n) windows [i, i+5) of an (F, n) MFCC sequence, R = F - 5."""
    m = np.asarray(mfcc, np.float64)
    R = len(m) - 5
    return np.stack([m[d:d + R] for d in range(5)], axis=1)


def feature_bound(win, ref_rows):
    """Elementwise first-order bound on |device row - reference row| (module doc)."""
    n = win.shape[2]
    E = U_MFCC * np.linalg.norm(win, axis=2).max(axis=1, keepdims=True)  # (R, 1)
    std = win.std(axis=1)  # (R, n)
    mn = np.abs(np.nan_to_num(ref_rows[:, :n]))
    with np.errstate(divide="ignore"):
        b_mn = ELEM_C * 2 * E * (1 + mn) / std
    b_d1 = np.broadcast_to(ELEM_C * 2 * E, (len(win), n))
    b_d2 = ELEM_C * 2 * E + 2 * b_mn
    return np.concatenate([b_mn, b_d1, b_d2], axis=1)


def flat_nan_mask(win):
    """Elements the reference formula makes 0/0: a coefficient constant over
    the window gives NaN in Mn and in D2 (D1 stays finite)."""
    flat = win.max(axis=1) == win.min(axis=1)
    return np.concatenate([flat, np.zeros_like(flat), flat], axis=1)


def check_rows(got, ref, win, name, row_frac=1.0):
    """NaN positions exact, elementwise bound everywhere, per-row ROW_TOL on
    at least row_frac of the rows; returns (worst row rel, its index)."""
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    assert got.shape == ref.shape, (got.shape, ref.shape)
    np.testing.assert_array_equal(np.isnan(got), np.isnan(ref), err_msg=f"{name}: NaN positions")
    fin = ~np.isnan(ref)
    d = np.where(fin, np.abs(got - ref), 0.0)
    bound = feature_bound(win, ref)
    over = fin & ~(d <= bound)
    assert not over.any(), (name, np.argwhere(over)[:5], d[over][:5], bound[over][:5])
    ok_rows = fin.all(axis=1)
    rel = np.linalg.norm(d[ok_rows], axis=1) / np.linalg.norm(ref[ok_rows], axis=1)
    frac = float((rel <= ROW_TOL).mean())
    worst = float(rel.max())
    print(f"{name}: {ok_rows.sum()} finite rows, worst row rel {worst:.3e} "
          f"(row {int(np.nonzero(ok_rows)[0][rel.argmax()])}), rows within {ROW_TOL:g}: {frac:.5f}")
    assert frac >= row_frac, (name, frac)
    return worst


def _ref39(w):
    return [(w[f"ref39_W{i}"], w[f"ref39_b{i}"]) for i in range(4)]


def _record(tmp_path, golden, key_frames, key_rows, key_returns):
    from vad_amd.sklearn_analyser import SKLearnAnalyzer
    g = golden("analyser")
    ref_rows = g[key_rows]
    labels = O.ffn_labels(ref_rows, _ref39(golden("ffn")))
    p = tmp_path / f"rec_{key_frames}.pkl"
    with open(p, "wb") as f:
        pickle.dump(FeatureRecorder(labels), f)
    an = SKLearnAnalyzer(str(p))
    an.load_init_inactive_frames(list(g["noise"]))
    frames = list(g[key_frames])
    rets = []
    for fr in frames:
        r = an.feed_frame(fr)
        rets.append(-1 if r is None else next(i for i, s in enumerate(frames) if s is r))
    np.testing.assert_array_equal(rets, g[key_returns])
    rows = np.concatenate(an.classifier.rows)
    assert rows.dtype == np.float64 and rows.shape == ref_rows.shape
    fb = O.get_mel_filterbanks(300, 8000, 512, 26, 16000)
    mfcc = np.stack([O.get_mfcc(fr, 512, fb, 13) for fr in frames])  # fp64 oracle: the reference's to 1e-12
    return rows, ref_rows, windows(mfcc)


@pytest.mark.parametrize("key", ["stream", "blocks"])
def test_analyser_rows_match_reference_run(torch_cuda, golden, tmp_path, key):
    """Every (1, 39) row the drop-in analyser passes to predict vs the row the
    reference passed on the same calls (stream: 193 rows incl. 9 silent
    windows; blocks: vad.py's 800-value blocks, truncated by the 512-pt FFT)."""
    rows_key = "features" if key == "stream" else "features_blocks"
    ret_key = "returns" if key == "stream" else "returns_blocks"
    got, ref, win = _record(tmp_path, golden, key, rows_key, ret_key)
    if key == "stream":
        # digital silence: all 13 Mn and all 13 D2 NaN in the reference run
        silent = np.isnan(ref).any(axis=1)
        assert silent.sum() == 9 and np.isnan(ref[silent][:, :13]).all() and np.isnan(ref[silent][:, 26:]).all()
        np.testing.assert_array_equal(np.isnan(ref), flat_nan_mask(win))
    check_rows(got, ref, win, f"analyser rows ({key})")


@pytest.mark.parametrize("fbank_num,low_hz,high_hz", [(40, 300, 8000), (20, 100, 7000)])
def test_analyser_rows_other_banks_vs_oracle(torch_cuda, golden, tmp_path, fbank_num, low_hz, high_hz):
    """The analyser's constructor parameters beyond the reference defaults
    (sklearn_analyser.py:16-33: fbank_num, low_hz, high_hz): the compiled
    40-filter bank and a runtime-table bank (20 filters, 100-7000 Hz), rows
    passed to predict vs the oracle's rows of the oracle's fp64 MFCCs on the
    fixture stream (parity pinned through the oracle's filterbank and MFCC
    fixtures; the reference run covers the 26-filter default only)."""
    from vad_amd.sklearn_analyser import SKLearnAnalyzer
    g = golden("analyser")
    frames = list(g["stream"])
    p = tmp_path / "rec.pkl"
    with open(p, "wb") as f:
        pickle.dump(FeatureRecorder([0] * len(frames)), f)
    an = SKLearnAnalyzer(str(p), low_hz=low_hz, high_hz=high_hz, fbank_num=fbank_num)
    an.load_init_inactive_frames(list(g["noise"]))
    for fr in frames:
        an.feed_frame(fr)
    got = np.concatenate(an.classifier.rows)
    fb = O.get_mel_filterbanks(low_hz, high_hz, 512, fbank_num, 16000)
    mfcc = np.stack([O.get_mfcc(fr, 512, fb, 13) for fr in frames])
    win = windows(mfcc)
    ref = np.where(flat_nan_mask(win), np.nan, O.analyser_features(mfcc))
    assert got.shape == ref.shape == (len(frames) - 5, 39)
    check_rows(got, ref, win, f"analyser rows ({fbank_num} filters, {low_hz}-{high_hz} Hz)")


def test_c3_clip_features_vs_oracle(torch_cuda):
    """C3 size (1M frames): the device's analyser window features vs the
    oracle's features of the oracle's fp64 MFCCs, NaN positions exact (flat
    coefficients), elementwise bound everywhere."""
    torch = torch_cuda
    from vad_amd.pipeline import VadPipeline
    from vad_amd.plan import window_features
    F = 1_000_000
    clip = O.synth_clip(O.samples_for_frames(F), seed=1)
    m = VadPipeline().mfcc(torch.from_numpy(clip).cuda())
    got = window_features(m).cpu().numpy()
    del m
    fb = O.get_mel_filterbanks(300, 8000, 512, 26, 16000)
    chunk = 100_000
    ref_m = np.concatenate([O.mfcc_batch(clip[160 * f0: 160 * (min(F, f0 + chunk) - 1) + 401], fb)
                            for f0 in range(0, F, chunk)])
    win = windows(ref_m)
    ref = O.analyser_features_fast(ref_m)
    # the oracle's fp64 mean of five equal values can round (x - mean != 0):
    # the reference formula's 0/0 is what the reference run shows (fixture
    # test above) and what the device gives
    nanm = flat_nan_mask(win)
    assert nanm.any()  # digital silence exercised
    ref = np.where(nanm, np.nan, ref)
    check_rows(got, ref, win, "C3 window features", row_frac=0.995)


def test_tree_analyser_on_reference_rows(torch_cuda, golden, tmp_path):
    """GPU tree analyser (SKLearnAnalyzer with the fixture's node table) on the
    fixture stream: each call's return equals the one the tree gives on the
    REFERENCE row of that call (sklearn's double comparison), wherever the
    row's decision path clears every threshold by more than the feature bound."""
    from vad_amd.sklearn_analyser import SKLearnAnalyzer
    from vad_amd.tree import TreeClassifier
    gt = golden("tree")
    g = golden("analyser")
    tree = {k: gt[k] for k in ("feature", "threshold", "left", "right", "leaf", "nan_left", "classes")}
    tree["n_features"] = int(gt["n_features"])
    t = TreeClassifier(tree["feature"], tree["threshold"], tree["left"], tree["right"], tree["leaf"],
                       tree["nan_left"], tree["classes"], tree["n_features"])
    p = tmp_path / "tree.npz"
    t.save(str(p))
    an = SKLearnAnalyzer(str(p))
    assert isinstance(an.classifier, TreeClassifier)
    an.load_init_inactive_frames(list(g["noise"]))
    frames = list(g["stream"])
    rets = []
    for fr in frames:
        r = an.feed_frame(fr)
        rets.append(-1 if r is None else next(i for i, s in enumerate(frames) if s is r))
    rets = np.asarray(rets)
    ref_rows = g["features"]
    pred = O.tree_predict(tree, ref_rows)
    fb = O.get_mel_filterbanks(300, 8000, 512, 26, 16000)
    win = windows(np.stack([O.get_mfcc(fr, 512, fb, 13) for fr in frames]))
    bound = feature_bound(win, ref_rows)
    # decision path of each reference row: does it pass within the bound of a threshold?
    near = np.zeros(len(ref_rows), bool)
    for i, x in enumerate(ref_rows):
        node = 0
        while tree["feature"][node] >= 0:
            f = tree["feature"][node]
            v = x[f]
            if np.isnan(v):
                node = tree["left"][node] if tree["nan_left"][node] else tree["right"][node]
                continue
            if abs(v - tree["threshold"][node]) <= bound[i, f]:
                near[i] = True
            node = tree["left"][node] if np.float32(v) <= tree["threshold"][node] else tree["right"][node]
    want = np.full(len(frames), -1)
    for i in range(len(ref_rows)):
        call = i + 5
        if pred[i] == 1:
            want[call] = call - 3
    print(f"tree analyser: {int(near.sum())} of {len(ref_rows)} rows pass within the feature bound of a threshold")
    sure = np.concatenate([np.ones(5, bool), ~near])
    np.testing.assert_array_equal(rets[sure], want[sure])
    assert (pred == 1).any() and (pred == 0).any()  # both dispatch branches exercised
