"""The oracle against the reference's own outputs on seeded random inputs
(tests/golden/random.npz, written by tests/golden/gen_random.py from the
unmodified reference): mel banks over random parameters bit for bit, spectra
and MFCCs of random-length frames at random FFT lengths, and the analyser's
feed_frame returns and predict rows over streams of random-length frames."""
import os
import sys

import numpy as np
import pytest

from oracle import vad_oracle as O

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
from gen_random import bank_digest  # noqa: E402


@pytest.fixture(scope="module")
def rnd(golden):
    return golden("random")


def frame_list(flat, lens):
    offs = np.concatenate([[0], np.cumsum(lens)])
    return [flat[offs[i]:offs[i + 1]] for i in range(len(lens))]


def test_oracle_banks_bit_exact(rnd):
    import warnings
    for (lo, hi, fft_n, nf, sr), dig, shp in zip(rnd["bank_params"], rnd["bank_digests"], rnd["bank_shapes"]):
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            fb = O.get_mel_filterbanks(lo, hi, int(fft_n), int(nf), int(sr))
        assert fb.shape == tuple(shp)
        assert bank_digest(fb) == str(dig), (lo, hi, fft_n, nf, sr)


def test_oracle_frames(rnd):
    p = rnd["frame_params"]
    frames = frame_list(rnd["frames"], p[:, 6].astype(int))
    s_off = np.concatenate([[0], np.cumsum(p[:, 2].astype(int) // 2)])
    m_off = np.concatenate([[0], np.cumsum(p[:, 5].astype(int))])
    for i, (lo, hi, fft_n, nf, sr, mfcc_n, _) in enumerate(p):
        fft_n, nf, mfcc_n = int(fft_n), int(nf), int(mfcc_n)
        fb = O.get_mel_filterbanks(lo, hi, fft_n, nf, int(sr))
        spec = O.get_spec_mag(frames[i], fft_n)
        np.testing.assert_array_equal(spec, rnd["specs"][s_off[i]:s_off[i + 1]])
        m = O.get_mfcc(frames[i], fft_n, fb, mfcc_n)
        ref = rnd["mfccs"][m_off[i]:m_off[i + 1]]
        assert np.abs(m - ref).max() <= 1e-12 * np.abs(ref).max(), i


def test_oracle_analyser_streams(rnd, golden):
    w = golden("ffn")
    lay = [(w[f"ref39_W{i}"], w[f"ref39_b{i}"]) for i in range(4)]

    class Rec:
        def __init__(self):
            self.x = []

        def predict(self, x):
            self.x.append(np.array(x, np.float64).reshape(-1))
            return O.ffn_labels(np.asarray(x, np.float64), lay)

    for s in range(3):
        stream = frame_list(rnd[f"stream{s}_frames"], rnd[f"stream{s}_lens"])
        noise = frame_list(rnd[f"stream{s}_noise"], rnd[f"stream{s}_noise_lens"])
        rec = Rec()
        an = O.AnalyserOracle(rec)
        an.load_init_inactive_frames(noise)
        ids = {id(f): i for i, f in enumerate(stream)}
        rets = []
        for f in stream:
            r = an.feed_frame(f)
            rets.append(-1 if r is None else ids[id(r)])
        np.testing.assert_array_equal(rets, rnd[f"stream{s}_returns"])
        rows, ref = np.asarray(rec.x), rnd[f"stream{s}_rows"]
        assert rows.shape == ref.shape
        np.testing.assert_array_equal(np.isnan(rows), np.isnan(ref))
        ok = ~np.isnan(ref)
        assert np.abs(rows[ok] - ref[ok]).max() <= 1e-9 * max(1.0, np.abs(ref[ok]).max())
