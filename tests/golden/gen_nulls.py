"""Spectral-null fixture (tests/golden/nulls.npz): frames built on the
cyclotomic structure of the 512-point DFT, run through the UNMODIFIED
reference mfcc.py (verdict r05 item 5).

A 400-sample frame x (float32 values are rationals) has X[k] = 0 exactly iff
its polynomial P(z) = sum x[n] z^n vanishes at w^k, w = exp(-2 pi i / 512), a
primitive m-th root of unity with m = 512 / gcd(k, 512); a rational
polynomial vanishing there is divisible by the cyclotomic polynomial
Phi_m (z^(m/2) + 1 for m = 2^j >= 2).  The frames here are products of
those factors (impulse combs: z^256 + 1 nulls every odd bin, z^128 + 1 every
bin = 2 mod 4, z^64 + 1 every bin = 4 mod 8, ...), times a few shifts and
signs, all within 400 samples -- the exact nulls a reference-configuration
frame can have.  tests/test_oracle_golden.py proves from the filterbanks that
no filter of the 26- or 40-filter bank at 512 points can have ALL its taps
on null bins (the degrees of the cyclotomic factors it would need exceed
399), so every mel energy of these frames is a signal's, not the FFT's
rounding noise: the device must match the reference within the MFCC rule on
every frame (tests/test_gpu_parity.py::test_spectral_null_frames).

Recorded: frames (float32), the reference's get_spec_mag spectrum (its own
numpy FFT), its get_mfcc at 26 and 40 filters, and which bins are exact
nulls (from the factorisation, not from the FFT).

    python tests/golden/gen_nulls.py      (needs /root/reference)
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from gen_golden import FloorInt, import_reference  # noqa: E402


def comb_frames():
    """(frame, null-bin mask) pairs: products of z^(m/2) + 1 factors (and the
    z^(m/2) - 1 = prod of lower cyclotomics forms), scaled and shifted."""
    def poly(*halves, sign=+1):
        p = np.ones(1)
        for h in halves:
            f = np.zeros(h + 1)
            f[0] = 1.0
            f[h] = float(sign)
            p = np.convolve(p, f)
        return p
    # (256, 128, 8): degree 392 -- nulls bins 30..33, ALL the taps of filter 9
    # of the 40-filter bank (the one filter of the reference banks whose
    # cyclotomic degree, 392, fits a 400-sample frame)
    specs = [((256, 128, 8), +1), ((256, 128, 8), -1), ((256, 128, 4, 2, 1), +1),
             ((256,), +1), ((128,), +1), ((64,), +1), ((256, 128), +1), ((256, 64), +1),
             ((256, 64, 32, 16, 8, 4, 2, 1), +1), ((128, 64, 32, 16, 8, 4, 2, 1), +1),
             ((128,), -1), ((256,), -1), ((64, 128), -1)]
    out = []
    for halves, sign in specs:
        p = poly(*halves, sign=sign)
        if len(p) > 400:
            continue
        for shift, amp in ((0, 1.0), (3, 32767.0), (400 - len(p), -3.0)):
            x = np.zeros(400)
            x[shift:shift + len(p)] = amp * p
            out.append(x.astype(np.float32))
    return out


def exact_null_bins(frame, fft_n=512):
    """Bins k < fft_n/2 where the exact DFT of the (integer-valued) frame is
    0: integer polynomial evaluation at w^k in exact cyclotomic arithmetic,
    reduced with the power-of-two modulus z^(m/2) = -1."""
    x = np.rint(frame.astype(np.float64)).astype(np.int64)
    assert np.array_equal(x, frame), "integer-valued frames only"
    nulls = np.zeros(fft_n // 2, bool)
    for k in range(fft_n // 2):
        g = np.gcd(k, fft_n)
        m = fft_n // g
        if m == 1:
            nulls[k] = x.sum() == 0
            continue
        # w^k is a primitive m-th root r; r^n depends on n k mod fft_n; in
        # Z[r] with r^(m/2) = -1 the basis is r^0 .. r^(m/2 - 1)
        h = m // 2
        c = np.zeros(h, np.int64)
        for n, v in enumerate(x):
            if v:
                e = (n * (k // g)) % m  # r = w^g primitive: w^(k n) = r^((k/g) n)
                c[e % h] += v if e < h else -v
        nulls[k] = not c.any()
    return nulls


def main():
    mfcc, _, _ = import_reference()
    fft_n = FloorInt(512)
    frames = comb_frames()
    spec = np.stack([mfcc.get_spec_mag(f, fft_n) for f in frames])
    out = {"frames": np.stack(frames), "spec": spec,
           "null_bins": np.stack([exact_null_bins(f) for f in frames])}
    for nf in (26, 40):
        fb = mfcc.get_mel_filterbanks(300, 8000, fft_n, nf, 16000)
        out[f"mfcc{nf}"] = np.stack([mfcc.get_mfcc(f, fft_n, fb, 13) for f in frames])
    np.savez_compressed(os.path.join(HERE, "nulls.npz"), **out)
    print({k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
