"""Randomised golden vectors from the UNMODIFIED reference (tests/golden/random.npz).

Run:  python tests/golden/gen_random.py            (needs /root/reference)

gen_golden.py pins the oracle on fixed, hand-picked inputs.  This script
draws seeded random inputs over the parameter space the reference functions
accept and records the reference's own outputs (imported with the same shims
as gen_golden.py), so the tests can check the oracle and the device on them:

  banks     get_mel_filterbanks(low, high, fft_n, n_filters, rate) for random
            parameters (fft_n 64..2048, 2..48 filters): a SHA-256 of each
            float64 bank (NaN written as -7.0) and its shape -- the banks
            themselves would be megabytes
  frames    get_spec_mag / get_mfcc of frames of random length (1..1200) and
            amplitude, at fft_n 512 and random lengths, with a random finite
            bank and a random MFCC count
  streams   SKLearnAnalyzer.feed_frame over three streams of frames of random
            lengths (the 512-point FFT pads or truncates each), classified
            with the ref39 fixture network: returns and the rows handed to
            predict
"""
from __future__ import annotations

import hashlib
import os
import pickle
import sys
import tempfile
import warnings

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from gen_golden import FloorInt, import_reference  # noqa: E402
from oracle import vad_oracle as O  # noqa: E402

RATES = (8000, 16000, 22050, 44100)


def bank_digest(fb):
    a = np.ascontiguousarray(np.nan_to_num(np.asarray(fb, np.float64), nan=-7.0))
    return hashlib.sha256(a.tobytes()).hexdigest()


def draw_bank_params(rng):
    sr = int(rng.choice(RATES))
    lo = float(rng.uniform(0.0, 1500.0))
    hi = float(lo + rng.uniform(0.2, 1.0) * (sr / 2 - lo))
    return lo, hi, int(rng.integers(64, 2049)), int(rng.integers(2, 49)), sr


def main():
    mfcc, sa, _ = import_reference()
    rng = np.random.default_rng(20261018)
    out = {}
    warnings.simplefilter("ignore")

    # ---------------- banks ----------------
    params, digests, shapes = [], [], []
    for _ in range(80):
        lo, hi, fft_n, nf, sr = draw_bank_params(rng)
        fb = np.asarray(mfcc.get_mel_filterbanks(lo, hi, FloorInt(fft_n), nf, sr), np.float64)
        params.append((lo, hi, fft_n, nf, sr))
        digests.append(bank_digest(fb))
        shapes.append(fb.shape)
    out["bank_params"] = np.array(params, np.float64)
    out["bank_digests"] = np.array(digests)
    out["bank_shapes"] = np.array(shapes, np.int64)

    # ---------------- frames ----------------
    fparams, frames, specs, mfccs = [], [], [], []
    while len(frames) < 120:
        lo, hi, fft_n, nf, sr = draw_bank_params(rng)
        if rng.random() < 0.5:
            fft_n = 512
        fb = np.asarray(mfcc.get_mel_filterbanks(lo, hi, FloorInt(fft_n), nf, sr), np.float64)
        if not np.isfinite(fb).all() or (fb.sum(axis=1) == 0).any():
            continue
        mfcc_n = int(rng.integers(1, min(13, nf) + 1))
        L = int(rng.integers(1, 1201))
        fr = (rng.standard_normal(L) * 10.0 ** rng.uniform(-1, 4.3)).astype(np.float32)
        spec = np.asarray(mfcc.get_spec_mag(fr, FloorInt(fft_n)))
        m = np.asarray(mfcc.get_mfcc(fr, FloorInt(fft_n), fb, mfcc_n), np.float64)
        fparams.append((lo, hi, fft_n, nf, sr, mfcc_n, L))
        frames.append(fr)
        specs.append(spec.astype(np.float32))
        mfccs.append(m)
    out["frame_params"] = np.array(fparams, np.float64)
    out["frames"] = np.concatenate(frames)
    out["specs"] = np.concatenate(specs)
    out["mfccs"] = np.concatenate(mfccs)

    # ---------------- analyser streams ----------------
    w = np.load(os.path.join(HERE, "ffn.npz"))
    lay = [(w[f"ref39_W{i}"], w[f"ref39_b{i}"]) for i in range(4)]

    class Recorder:
        def __init__(self):
            self.x = []

        def predict(self, x):
            self.x.append(np.array(x, np.float64).reshape(-1))
            return O.ffn_labels(np.asarray(x, np.float64), lay)

    tmp = tempfile.mkdtemp()
    pkl = os.path.join(tmp, "clf.pkl")
    with open(pkl, "wb") as f:
        pickle.dump(None, f)
    for s in range(3):
        lens = rng.integers(1, 1001, 40)
        stream = [(rng.standard_normal(int(n)) * 10.0 ** rng.uniform(0, 4)).astype(np.float32) for n in lens]
        for i in rng.choice(40, 6, replace=False):
            stream[i][:] = 0.0  # digital silence: NaN rows
        noise = [(rng.standard_normal(int(n)) * 10.0).astype(np.float32) for n in rng.integers(1, 800, 5)]
        rec = Recorder()
        an = sa.SKLearnAnalyzer(pkl, fft_n=FloorInt(512))
        an.classifier = rec
        an.load_init_inactive_frames(list(noise))
        ids = {id(f): i for i, f in enumerate(stream)}
        rets = []
        for f in stream:
            r = an.feed_frame(f)
            rets.append(-1 if r is None else ids[id(r)])
        out[f"stream{s}_lens"] = np.asarray(lens, np.int64)
        out[f"stream{s}_frames"] = np.concatenate(stream)
        out[f"stream{s}_noise_lens"] = np.asarray([len(n) for n in noise], np.int64)
        out[f"stream{s}_noise"] = np.concatenate(noise)
        out[f"stream{s}_returns"] = np.asarray(rets, np.int64)
        out[f"stream{s}_rows"] = np.asarray(rec.x)
    np.savez_compressed(os.path.join(HERE, "random.npz"), **out)
    print("banks", len(digests), "frames", len(frames), "streams 3; size",
          os.path.getsize(os.path.join(HERE, "random.npz")), "bytes")


if __name__ == "__main__":
    main()
