"""Drop-in mirror of the reference ``mfcc.py`` module (same function names,
arguments and return types), backed by the HIP kernels.

The filterbank construction (mfcc.py:5-56) is one-off host setup in fp64,
restated here exactly as the reference computes it; the per-frame functions
(get_spec_mag, get_mfcc, get_mfcc_from_spec) run on the GPU through a plan
cache.  Frames are NumPy arrays in and out, as in the reference.
"""
from __future__ import annotations

import numpy as np
import torch

from .plan import MfccPlan

_EPS = np.finfo(float).eps


def mel_from_hz(first_hz, upper_hz, n_bins):
    """mfcc.py:5-18"""
    first_mel = 1125.0 * np.log(1.0 + first_hz / 700.0)
    last_mel = 1125.0 * np.log(1.0 + upper_hz / 700.0)
    delta = (last_mel - first_mel) / (n_bins + 1)
    mels = [first_mel + i * delta for i in range(n_bins + 1)]
    mels.append(last_mel)
    mels.sort()
    return mels


def one_hz_from_mel(mel):
    """mfcc.py:21-22"""
    return 700 * (np.exp(mel / 1125) - 1)


def hz_from_mel(mels):
    """mfcc.py:25-27"""
    return list(map(one_hz_from_mel, mels))


def convert_to_fft_bins(sample_rate, hzs, fft_n):
    """mfcc.py:30-36 (note fft_n + 1)"""
    return [np.floor((fft_n + 1) * hz / sample_rate) for hz in hzs]


def get_mel_filterbanks(low_hz, up_hz, fft_n, n_filters, sample_rate):
    """mfcc.py:39-56 -- (n_filters, fft_n // 2) float64 triangular filterbank."""
    hzs = hz_from_mel(mel_from_hz(low_hz, up_hz, n_filters))
    b = np.asarray(convert_to_fft_bins(sample_rate, hzs, fft_n), dtype=np.float64)
    half = int(fft_n) // 2
    k = np.arange(0, half, 1, dtype=np.float64)
    fb = np.zeros((n_filters, half))
    with np.errstate(divide="ignore", invalid="ignore"):
        for m in range(1, n_filters + 1):
            rise = (k >= b[m - 1]) & (k <= b[m])          # :50 (wins at k == b[m])
            fall = (~rise) & (k >= b[m]) & (k <= b[m + 1])  # :53 elif
            fb[m - 1, rise] = (k[rise] - b[m - 1] + 0.0) / (b[m] - b[m - 1] + 0.0)
            fb[m - 1, fall] = (b[m + 1] - k[fall] + 0.0) / (b[m + 1] - b[m] + 0.0)
    return fb


# ---------------------------------------------------------------------------
# per-frame functions on the GPU
# ---------------------------------------------------------------------------
_plans = {}


def plan_for(filterbank, mfcc_n=13, fft_n=512):
    """Cached MfccPlan for a filterbank array (keyed by its bytes)."""
    fb = np.ascontiguousarray(np.asarray(filterbank, dtype=np.float64))
    key = (fb.shape, fb.tobytes(), int(mfcc_n), int(fft_n))
    p = _plans.get(key)
    if p is None:
        p = MfccPlan(fb, mfcc_n, fft_n)
        _plans[key] = p
    return p


_spec_plans = {}


def _frame_tensor(frame):
    x = np.ascontiguousarray(np.asarray(frame).astype(np.float32).reshape(-1))
    if x.size == 0:
        raise ValueError("empty frame")
    return torch.from_numpy(x).cuda()


def get_spec_mag(frame, fft_n=512):
    """mfcc.py:59-61 -- |fft(frame, fft_n)[:fft_n/2] / fft_n|^2 as float32 (fft_n // 2,).

    fft_n = 512 (the reference's only value) runs the radix-16 kernels, any
    other length (2..8192) a direct DFT with fp64 accumulation."""
    n = int(fft_n)
    p = _spec_plans.get(n)
    if p is None:
        p = _spec_plans[n] = MfccPlan(get_mel_filterbanks(300, 8000, n, 26, 16000), 13, n)
    x = _frame_tensor(frame)
    return p.spec(x, frame_len=x.numel(), frame_stride=x.numel(), n=1)[0].cpu().numpy()


def get_mfcc(frame, fft_n, filterbank, mfcc_n):
    """mfcc.py:67-69 -- MFCCs of one frame, float64 (mfcc_n,)."""
    x = _frame_tensor(frame)
    p = plan_for(filterbank, mfcc_n, fft_n)
    return p.mfcc(x, frame_len=x.numel(), frame_stride=x.numel(), n=1)[0].cpu().numpy().astype(
        np.float64)


def get_mfcc_from_spec(spec, filterbank, mfcc_n):
    """mfcc.py:72-78 -- MFCCs of one (B,) spectrum (or a (n, B) batch), float64;
    B = the filterbank's columns (256 for the reference's fft_n = 512)."""
    s = np.ascontiguousarray(np.asarray(spec, dtype=np.float32))
    single = s.ndim == 1
    t = torch.from_numpy(s.reshape(-1, s.shape[-1])).cuda()
    fb = np.asarray(filterbank)
    out = plan_for(fb, mfcc_n, 2 * fb.shape[1]).from_spec(t).cpu().numpy().astype(np.float64)
    return out[0] if single else out


def get_deltas(mfcc2, mfcc1):
    """mfcc.py:81-82"""
    return np.subtract(mfcc2, mfcc1)


def lifter(cepstra, L=22):
    """mfcc.py:85-93 (folded into the DCT matrix inside the kernels)."""
    if L > 0:
        ncoeff = np.shape(cepstra)[0]
        n = np.arange(ncoeff)
        lift = 1 + (L / 2.) * np.sin(np.pi * n / L)
        return lift * cepstra
    return cepstra
