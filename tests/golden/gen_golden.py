"""Generate the golden fixtures in tests/golden/ by running the UNMODIFIED
reference (nameofuser1/vad at /root/reference) in the build container.

Run:  python tests/golden/gen_golden.py            (needs /root/reference)

The reference is Python 2 code; it is imported unmodified with three
import-time shims: the module search path, ``cPickle`` ->
``pickle`` (sklearn_analyser.py:1) and ``h5py`` stubbed (only the file-index
helpers of dataset/file_index.py use it).  ``fft_n`` is passed as an int
subclass whose ``/`` floors, because mfcc.py:45-46,61 use Py2 integer
division as an index.  The reference cannot travel to the GPU box; only the
arrays written here do (inputs and the reference's outputs).

FFN weights: the reference never committed any, so seeded
synthetic weights are drawn here, calibrated (final bias) to give mixed
labels, and the labels come from the oracle's fp64 restatement of
learning/ffn_trainer.py:106-116.
"""
from __future__ import annotations

import os
import pickle
import queue
import sys
import tempfile
import types

import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

from oracle import vad_oracle as O  # noqa: E402


class FloorInt(int):
    """Py2 '/' on ints (mfcc.py:45-46,61 index with fft_n/2)."""

    def __truediv__(self, o):
        return FloorInt(int(self) // o)


def import_reference():
    sys.path.insert(0, REF)
    sys.path.insert(0, os.path.join(REF, "realtime_analysis"))
    sys.modules.setdefault("cPickle", pickle)
    sys.modules.setdefault("h5py", types.ModuleType("h5py"))
    cwd = os.getcwd()
    os.chdir(tempfile.mkdtemp())  # sklearn_analyser.py:10 opens analyser.log at import
    try:
        import mfcc  # noqa: F401
        import sklearn_analyser  # noqa: F401
        sys.path.append(os.path.join(REF, "dataset"))
        import file_processing  # noqa: F401
    finally:
        os.chdir(cwd)
    import logging
    logging.getLogger("sklearn_analyser").setLevel(logging.INFO)  # skip eager debug strings
    return sys.modules["mfcc"], sys.modules["sklearn_analyser"], sys.modules["file_processing"]


# --------------------------------------------------------------------------
# inputs
# --------------------------------------------------------------------------
def edge_frames(rng, n=400):
    t = np.arange(n, dtype=np.float64)
    fr = []
    fr.append(np.zeros(n))                                   # digital silence
    fr.append(np.full(n, 32767.0))                           # DC full scale
    fr.append(np.full(n, -1.0))                              # DC tiny
    fr.append(32767.0 * (-1.0) ** t)                         # alternating
    imp = np.zeros(n); imp[0] = 32767.0; fr.append(imp)      # impulse first
    imp = np.zeros(n); imp[n - 1] = 1.0; fr.append(imp)      # impulse last, tiny
    imp = np.zeros(n); imp[200] = -5.0; fr.append(imp)
    for f0 in (62.5, 1000.0, 1031.25, 3999.0, 7968.75, 300.0, 8000.0):
        fr.append(np.rint(20000.0 * np.sin(2 * np.pi * f0 * t / 16000.0)))
    fr.append(np.linspace(-32767, 32767, n).round())          # ramp
    for a in (1.0, 3.0, 10.0, 100.0, 1000.0, 10000.0, 40000.0):
        fr.append(np.clip(np.rint(a * rng.standard_normal(n)), -32767, 32767))
    fr.append(rng.uniform(-1.0, 1.0, n))                      # non-integer floats
    fr.append(rng.uniform(-1e-3, 1e-3, n))
    one = np.zeros(n); one[137] = 1.0; one[138] = 1.0; fr.append(one)
    return np.asarray(fr, np.float32)


def main():
    mfcc, sa, fp = import_reference()
    rng = np.random.default_rng(20261015)
    fft_n = FloorInt(512)
    out = {}

    # ---------------- filterbanks (mfcc.py:39-56) ----------------
    fbs = {
        "fb_26": (300, 8000, 26, 16000),
        "fb_40": (300, 8000, 40, 16000),
        "fb_20_0_8000": (0, 8000, 20, 16000),
        "fb_32_100_4000": (100, 4000, 32, 16000),
    }
    fbd = {}
    for name, (lo, hi, nf, sr) in fbs.items():
        fbd[name] = mfcc.get_mel_filterbanks(lo, hi, fft_n, nf, sr)
        fbd[name + "_params"] = np.array([lo, hi, nf, sr], np.float64)
        hzs = mfcc.hz_from_mel(mfcc.mel_from_hz(lo, hi, nf))
        fbd[name + "_bins"] = np.asarray(mfcc.convert_to_fft_bins(sr, hzs, 512), np.float64)
    np.savez_compressed(os.path.join(HERE, "filterbanks.npz"), **fbd)
    fb26, fb40 = fbd["fb_26"], fbd["fb_40"]

    # ---------------- single frames (mfcc.py:59-78) ----------------
    clip = O.synth_clip(16000 * 4, seed=7)
    rand_frames = O.frame_matrix(clip)[rng.choice(O.n_frames(len(clip)), 200, replace=False)]
    frames = np.concatenate([edge_frames(rng), rand_frames.astype(np.float32)])
    spec = np.stack([mfcc.get_spec_mag(f, fft_n) for f in frames])
    m26 = np.stack([mfcc.get_mfcc_from_spec(s, fb26, 13) for s in spec])
    m40 = np.stack([mfcc.get_mfcc_from_spec(s, fb40, 13) for s in spec])
    # other frame lengths: truncation (>512, vad.py's 800-value int8 blocks) and short frames
    odd = {}
    for L in (800, 512, 256, 401):
        fr = np.clip(np.rint(300.0 * rng.standard_normal((6, L))), -127 if L == 800 else -32767,
                     127 if L == 800 else 32767).astype(np.float32)
        odd[f"frames_{L}"] = fr
        odd[f"spec_{L}"] = np.stack([mfcc.get_spec_mag(f, fft_n) for f in fr])
        odd[f"mfcc26_{L}"] = np.stack([mfcc.get_mfcc(f, fft_n, fb26, 13) for f in fr])
    np.savez_compressed(os.path.join(HERE, "frames.npz"), frames=frames, spec=spec,
                        mfcc26=m26, mfcc40=m40, n_edge=np.int64(len(edge_frames(rng))), **odd)

    # ---------------- framing + offline features (file_processing.py:14-103) -------
    lens = np.array([0, 1, 399, 400, 401, 559, 560, 561, 720, 721, 16000, 16241], np.int64)
    counts = np.array([len(fp.split_into_frames(np.zeros(L, np.int16), 400, 160)) for L in lens])
    clip16 = O.synth_clip(16000, seed=11).astype(np.int16)
    from scipy.io import wavfile
    tmp = tempfile.mkdtemp()
    wav = os.path.join(tmp, "clip.wav")
    wavfile.write(wav, 16000, clip16)
    q = queue.Queue()
    q.put(0)
    feats = fp.process_file((wav, 400, 160, fft_n, fb26, 13, q, None))
    feats = np.asarray([[np.asarray(a) for a in row] for row in feats], np.float64)
    clip_mfcc = np.stack([mfcc.get_mfcc(f, fft_n, fb26, 13)
                          for f in fp.split_into_frames(clip16, 400, 160)])
    np.savez_compressed(os.path.join(HERE, "clip.npz"), lens=lens, counts=counts,
                        clip=clip16, features=feats, mfcc=clip_mfcc)

    # ---------------- FFN weights (seeded, calibrated) --------------------
    def he_uniform(r, fan_in, fan_out):
        lim = np.sqrt(6.0 / fan_in)
        return r.uniform(-lim, lim, (fan_in, fan_out)).astype(np.float32)

    wr = np.random.default_rng(39)
    dims = [39, 64, 32, 16, 3]
    layers = [(he_uniform(wr, a, b), (0.05 * wr.standard_normal(b)).astype(np.float32))
              for a, b in zip(dims[:-1], dims[1:])]
    # calibration data: analyser features of a synthetic clip at a 10 ms hop
    cal_clip = O.synth_clip(16000 * 8, seed=3)
    cal_x = O.analyser_features(O.mfcc_batch(cal_clip, fb26))
    ok = ~np.isnan(cal_x).any(axis=1)
    z, _ = O.ffn_forward(cal_x[ok], layers)
    # centre logits so that classes 0/1 split ~evenly; class 2 (MUSIC) well below
    b4 = layers[-1][1].astype(np.float64)
    d01 = np.median(z[:, 1] - z[:, 0])
    z2 = z.copy()
    z2[:, 1] -= d01
    gap = z2[:, 2] - np.maximum(z2[:, 0], z2[:, 1])
    b4[1] -= d01
    b4m = b4.copy()
    b4[2] -= np.max(gap) + 1.0          # class 2 never wins on the calibration clip
    b4m[2] -= np.percentile(gap, 90)    # MUSIC variant: class 2 wins ~10% (AssertionError, :82)
    layers[-1] = (layers[-1][0], b4.astype(np.float32))
    # BASELINE.json config 3 topology 13 -> 64 -> 64 -> 2 on the normalised centre MFCC
    br = np.random.default_rng(13)
    bl = [(he_uniform(br, 13, 64), (0.05 * br.standard_normal(64)).astype(np.float32)),
          (he_uniform(br, 64, 64), (0.05 * br.standard_normal(64)).astype(np.float32)),
          (he_uniform(br, 64, 2), np.zeros(2, np.float32))]
    zb, _ = O.ffn_forward(cal_x[ok][:, :13], bl)
    bl[-1] = (bl[-1][0], np.array([0.0, -np.median(zb[:, 1] - zb[:, 0])], np.float32))

    test_clip = O.synth_clip(16000 * 6, seed=5)
    test_mfcc = O.mfcc_batch(test_clip, fb26)
    test_x = O.analyser_features(test_mfcc)
    wd = {}
    for i, (w, b) in enumerate(layers):
        wd[f"ref39_W{i}"], wd[f"ref39_b{i}"] = w, b
    wd["ref39_b3_music"] = b4m.astype(np.float32)
    for i, (w, b) in enumerate(bl):
        wd[f"bl13_W{i}"], wd[f"bl13_b{i}"] = w, b
    lay_m = layers[:-1] + [(layers[-1][0], b4m.astype(np.float32))]
    wd["test_clip"] = test_clip
    wd["test_x"] = test_x
    wd["test_labels_ref39"] = O.ffn_labels(test_x, layers)
    wd["test_margin_ref39"] = O.ffn_margin(test_x, layers)
    wd["test_labels_music"] = O.ffn_labels(test_x, lay_m)
    wd["test_labels_bl13"] = O.ffn_labels(test_x[:, :13], bl)
    wd["test_margin_bl13"] = O.ffn_margin(test_x[:, :13], bl)
    np.savez_compressed(os.path.join(HERE, "ffn.npz"), **wd)

    # ---------------- streaming analyser trace (sklearn_analyser.py) -------
    class Recorder:
        def __init__(self, lay):
            self.lay, self.x = lay, []

        def predict(self, x):
            self.x.append(np.array(x, np.float64).reshape(-1))
            return O.ffn_labels(np.asarray(x, np.float64), self.lay)

    def run_trace(lay, stream, noise, init=True):
        rec = Recorder(lay)
        pkl = os.path.join(tmp, "clf.pkl")
        with open(pkl, "wb") as f:
            pickle.dump(None, f)
        an = sa.SKLearnAnalyzer(pkl, fft_n=fft_n)
        an.classifier = rec
        if init:
            an.load_init_inactive_frames(list(noise))
        rets, err = [], ""
        ids = {id(f): i for i, f in enumerate(stream)}
        for i, f in enumerate(stream):
            try:
                r = an.feed_frame(f)
            except Exception as e:  # noqa: BLE001 - recorded, not swallowed
                err = f"{i}:{type(e).__name__}"
                break
            rets.append(-1 if r is None else ids[id(r)])
        x = np.asarray(rec.x) if rec.x else np.zeros((0, 39))
        return np.asarray(rets, np.int64), x, err

    sclip = O.synth_clip(16000 * 2, seed=21)
    sclip[4000:6000] = 0.0  # digital silence inside the stream -> NaN features
    stream = [f.copy() for f in O.frame_matrix(sclip)]     # 10 ms hop, 400-sample frames
    noise = [f.copy() for f in O.frame_matrix(O.synth_clip(2000, seed=22))[:5]]
    r, x, err = run_trace(layers, stream, noise)
    tr = {"stream": np.asarray(stream), "noise": np.asarray(noise), "returns": r,
          "features": x, "error": np.array(err)}
    r, x, err = run_trace(lay_m, stream, noise)
    tr.update(returns_music=r, features_music=x, error_music=np.array(err))
    blocks = [np.clip(np.rint(50 * rng.standard_normal(800)), -127, 127).astype(np.float32)
              for _ in range(12)]                               # vad.py's 800-value blocks
    r, x, err = run_trace(layers, blocks, noise)
    tr.update(blocks=np.asarray(blocks), returns_blocks=r, features_blocks=x,
              error_blocks=np.array(err))
    r, x, err = run_trace(layers, stream[:3], noise, init=False)
    tr.update(error_noinit=np.array(err))
    try:
        sa.SKLearnAnalyzer.load_init_inactive_frames(
            type("S", (), {"fft_n": fft_n})(), noise[:4])
        tr["error_badinit"] = np.array("")
    except Exception as e:  # noqa: BLE001
        tr["error_badinit"] = np.array(type(e).__name__)
    np.savez_compressed(os.path.join(HERE, "analyser.npz"), **tr)
    for k in ("returns", "returns_music", "returns_blocks"):
        print(k, "voiced:", int((tr[k] >= 0).sum()), "of", len(tr[k]))
    print("errors:", tr["error"], tr["error_music"], tr["error_blocks"], tr["error_noinit"],
          tr["error_badinit"])
    print("ffn test labels:", np.bincount(wd["test_labels_ref39"], minlength=3),
          "min margin", np.min(wd["test_margin_ref39"]))


if __name__ == "__main__":
    main()
