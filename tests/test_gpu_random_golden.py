"""The device path against the reference's own outputs on seeded random
inputs (tests/golden/random.npz, from tests/golden/gen_random.py): spectra
and MFCCs of random-length frames at random FFT lengths with random banks
(tolerances of tests/test_gpu_parity.py), and the drop-in SKLearnAnalyzer
(FFN .npz: the fused device step; and a pickled foreign classifier) replaying
the reference's streams of random-length frames: every return equal to the
reference's wherever the fp64 margin of the reference's own row for that
call exceeds MARGIN_TOL."""
import os
import pickle

import numpy as np
import pytest

from oracle import vad_oracle as O

pytestmark = pytest.mark.gpu

SPEC_TOL = 1e-5
MFCC_TOL = 1e-4
MARGIN_TOL = 0.05


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    return torch


def frame_list(flat, lens):
    offs = np.concatenate([[0], np.cumsum(lens)])
    return [flat[offs[i]:offs[i + 1]] for i in range(len(lens))]


def test_random_frames_vs_reference(torch_cuda, golden):
    from vad_amd import mfcc as M
    r = golden("random")
    p = r["frame_params"]
    frames = frame_list(r["frames"], p[:, 6].astype(int))
    s_off = np.concatenate([[0], np.cumsum(p[:, 2].astype(int) // 2)])
    m_off = np.concatenate([[0], np.cumsum(p[:, 5].astype(int))])
    for i, (lo, hi, fft_n, nf, sr, mfcc_n, _) in enumerate(p):
        fft_n, nf, mfcc_n = int(fft_n), int(nf), int(mfcc_n)
        fb = M.get_mel_filterbanks(lo, hi, fft_n, nf, int(sr))
        spec = M.get_spec_mag(frames[i], fft_n)
        ref_s = r["specs"][s_off[i]:s_off[i + 1]].astype(np.float64)
        nr = np.linalg.norm(ref_s)
        assert (np.abs(spec).max() == 0) if nr == 0 else np.linalg.norm(spec - ref_s) / nr <= SPEC_TOL, i
        m = M.get_mfcc(frames[i], fft_n, fb, mfcc_n)
        ref = r["mfccs"][m_off[i]:m_off[i + 1]]
        d = m - ref
        assert np.linalg.norm(d) / np.linalg.norm(ref) <= MFCC_TOL, i
        assert np.abs(d).max() / np.abs(ref).max() <= MFCC_TOL, i


@pytest.mark.parametrize("form", ["npz", "pickle"])
def test_random_streams_vs_reference(torch_cuda, golden, tmp_path, form):
    from vad_amd.ffn import save_layers
    from vad_amd.sklearn_analyser import SKLearnAnalyzer
    r = golden("random")
    w = golden("ffn")
    lay = [(w[f"ref39_W{i}"], w[f"ref39_b{i}"]) for i in range(4)]
    if form == "npz":
        path = tmp_path / "ffn.npz"
        save_layers(str(path), lay)
    else:
        path = tmp_path / "clf.pkl"
        with open(path, "wb") as f:
            pickle.dump(O.FFNPredictor(lay), f)
    n_checked = 0
    for s in range(3):
        stream = frame_list(r[f"stream{s}_frames"], r[f"stream{s}_lens"])
        noise = frame_list(r[f"stream{s}_noise"], r[f"stream{s}_noise_lens"])
        rows = r[f"stream{s}_rows"]
        want = r[f"stream{s}_returns"]
        an = SKLearnAnalyzer(str(path))
        an.load_init_inactive_frames(noise)
        ids = {id(f): i for i, f in enumerate(stream)}
        for i, f in enumerate(stream):
            got = an.feed_frame(f)
            g = -1 if got is None else ids[id(got)]
            if i < 5:
                assert g == -1 == want[i]
            elif O.ffn_margin(rows[i - 5][None], lay)[0] > MARGIN_TOL:
                assert g == want[i], (s, i, g, want[i])
                n_checked += 1
    assert n_checked > 0.8 * 3 * 35
