"""Optional pre-emphasis / Hamming stages (BASELINE north_star names them;
the reference has neither, mfcc.py:59-61): default off and then bit-identical
to the reference-parity path; on, equal to the oracle's restatement
(python_speech_features conventions) -- parity unpinned against the
reference, which has no output for them."""
import numpy as np
import pytest

from oracle import vad_oracle as O

pytestmark = pytest.mark.gpu

MFCC_TOL = 1e-4


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    return torch


def _close(got, ref, tol=MFCC_TOL):
    got, ref = np.asarray(got, np.float64), np.asarray(ref, np.float64)
    assert got.shape == ref.shape
    d = got - ref
    rel = np.linalg.norm(d, axis=1) / np.linalg.norm(ref, axis=1)
    mx = np.abs(d).max(axis=1) / np.abs(ref).max(axis=1)
    assert rel.max() <= tol and mx.max() <= tol, (rel.max(), mx.max())


def test_stages_off_is_bit_identical(torch_cuda):
    torch = torch_cuda
    from vad_amd.config import MfccConfig
    from vad_amd.pipeline import VadPipeline
    from vad_amd.plan import MfccPlan
    clip = torch.from_numpy(O.synth_clip(O.samples_for_frames(5000), seed=61)).cuda()
    base = VadPipeline().mfcc(clip)
    assert torch.equal(VadPipeline(cfg=MfccConfig(preemph=None, window=None)).mfcc(clip), base)
    # a window set and removed again leaves the plan's outputs unchanged
    p = MfccPlan.from_config(MfccConfig())
    v = p.variant
    p.set_window(np.hamming(400))
    assert p.variant == 3
    p.set_window(None)
    assert p.variant == v
    assert torch.equal(p.clip_mfcc(clip), base)


@pytest.mark.parametrize("preemph,window", [(None, "hamming"), (0.97, None), (0.97, "hamming")])
def test_stages_vs_oracle(torch_cuda, preemph, window):
    torch = torch_cuda
    from vad_amd.config import MfccConfig
    from vad_amd.ffn import TOPOLOGY_BL13, FFNClassifier, random_layers
    from vad_amd.pipeline import VadPipeline
    F = 20_000
    clip = O.synth_clip(O.samples_for_frames(F), seed=62)
    cfg = MfccConfig(preemph=preemph, window=window)
    layers = random_layers(TOPOLOGY_BL13, seed=3)
    pipe = VadPipeline(FFNClassifier(layers), cfg=cfg)
    a = torch.from_numpy(clip).cuda()
    m = pipe.mfcc(a).cpu().numpy()
    fb = O.get_mel_filterbanks(300, 8000, 512, 26, 16000)
    w = np.hamming(400) if window else None
    ref = O.mfcc_batch(clip, fb, preemph=preemph, window=w)
    _close(m, ref)
    # int16 PCM in: the same MFCCs
    assert np.array_equal(pipe.mfcc(a.to(torch.int16)).cpu().numpy(), m)
    # labels of the windowed / pre-emphasised clip (two-kernel form: a
    # windowed plan is not the fused kernel's compiled bank)
    assert not pipe.fusable or window is None
    lab = pipe.labels(a).cpu().numpy()
    x = O.analyser_features_fast(ref)[:, :13]
    sure = O.ffn_margin(x, layers) > 0.05
    np.testing.assert_array_equal(lab[sure], O.ffn_labels(x, layers)[sure])
    if window:  # spectra of the windowed frames
        fr = O.frame_matrix(O.preemphasis(clip, preemph) if preemph else clip)[:2000]
        spec = pipe.plan.spec(torch.from_numpy(np.ascontiguousarray(fr)).cuda()).cpu().numpy()
        ref_s = O.spec_batch(fr.astype(np.float32) * np.hamming(400).astype(np.float32))
        nz = np.linalg.norm(ref_s, axis=1) > 0
        rel = np.linalg.norm(spec[nz] - ref_s[nz], axis=1) / np.linalg.norm(ref_s[nz], axis=1)
        assert rel.max() <= 1e-5


def test_preemphasis_kernel(torch_cuda):
    torch = torch_cuda
    from vad_amd.plan import preemphasis
    x = O.synth_clip(100_003, seed=63)
    got = preemphasis(torch.from_numpy(x).cuda(), 0.95).cpu().numpy()
    np.testing.assert_array_equal(got, O.preemphasis(x, 0.95))  # same roundings
    rows = x[:400 * 7].reshape(7, 400)
    got2 = preemphasis(torch.from_numpy(rows.copy()).cuda(), 0.95).cpu().numpy()
    np.testing.assert_array_equal(got2, np.stack([O.preemphasis(r, 0.95) for r in rows]))
