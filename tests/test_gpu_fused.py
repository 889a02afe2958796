"""The fused clip kernel (vad_mfcc_ffn: MFCC -> window features -> FFN in one
launch, MFCC rows kept on chip) against the two-kernel form and the oracle.

Labels of the fused and the two-kernel path must be identical bit for bit
(same MFCC arithmetic, same features, same split-f16 forward): clip lengths
around every workgroup / tile / halo boundary, both specialised topologies and
a 3-class bl13, fp32 and int16 input, analyser and offline features.
"""
import numpy as np
import pytest

from oracle import vad_oracle as O

pytestmark = pytest.mark.gpu

TOPOS = ((13, 64, 64, 2), (39, 64, 32, 16, 3), (13, 64, 64, 3))
# F frames: a single partial tile, the first tile-edge windows, 256-workgroup
# splits with 1..2 tiles each, uneven splits, and multi-tile runs
FRAMES = (6, 7, 8, 64, 68, 69, 70, 133, 1000, 16_389, 16_389 + 257, 65_541, 100_003)


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    return torch


def _pipe(topo, mode="analyser"):
    from vad_amd.ffn import FFNClassifier, random_layers
    from vad_amd.pipeline import VadPipeline
    return VadPipeline(FFNClassifier(random_layers(topo, seed=3)), mode=mode)


@pytest.mark.parametrize("topo", TOPOS)
def test_fused_equals_two_kernel(torch_cuda, topo):
    torch = torch_cuda
    clip = O.synth_clip(O.samples_for_frames(max(FRAMES)), seed=21)
    clip[160 * 5000:160 * 5100] = 0.0  # digital silence: NaN windows -> class 0
    a32 = torch.from_numpy(clip).cuda()
    a16 = a32.round().clamp(-32768, 32767).to(torch.int16)
    for mode in ("analyser", "offline"):
        pipe = _pipe(topo, mode)
        assert pipe.fusable
        for F in FRAMES:
            n = O.samples_for_frames(F)
            for a in (a32[:n], a16[:n]):
                got = pipe.labels(a, fused=True)
                want = pipe.labels(a)
                assert got.numel() == F - 5
                assert torch.equal(got, want), (topo, mode, F, a.dtype,
                                                int((got != want).sum()))


def test_fused_independent_of_stale_lds(torch_cuda):
    """The fused kernel's first tile has no previous tile: ring rows 0..3
    (the halo of windows before the workgroup's first, never stored) share
    wave 0's 16-window tile with stored windows.  They are zeroed, not left
    as whatever an earlier kernel wrote to that LDS: stale values past f16
    range would force the tile's split-f16 rescale and perturb its real
    windows (found by tests/test_gpu_fuzz.py on a box whose LDS held such
    values).  Here a test-only kernel (tests/c_host/lds_poison.hip) fills
    every CU's 160 KB of LDS with 1e30 right before each fused launch; the
    fused labels must still equal the two-kernel labels, for short clips (one
    workgroup, its first tile only) in both feature forms."""
    import ctypes
    import os
    torch = torch_cuda
    so = os.path.join(os.path.dirname(os.path.abspath(__file__)), "c_host", "liblds_poison.so")
    if not os.path.exists(so):
        pytest.fail("tests/c_host/liblds_poison.so missing: run __graft_entry__.build()")
    helper = ctypes.CDLL(so)
    helper.lds_poison.argtypes = [ctypes.c_float, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    sink = torch.zeros(1, device="cuda")
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    n_cu = torch.cuda.get_device_properties(0).multi_processor_count
    for mode in ("analyser", "offline"):
        pipe = _pipe((39, 64, 32, 16, 3), mode)
        for F in (6, 9, 12, 21, 40, 70):
            for seed in range(3):
                rng = np.random.default_rng(100 * F + seed)
                clip = rng.standard_normal(O.samples_for_frames(F)).astype(np.float32)
                a = torch.from_numpy(clip).cuda()
                want = pipe.labels(a)
                assert helper.lds_poison(1e30, ctypes.c_void_p(sink.data_ptr()), 4 * n_cu, stream) == 0
                got = pipe.labels(a, fused=True)
                assert torch.equal(got, want), (mode, F, seed, got.tolist(), want.tolist())
    assert sink.item() == 0.0  # the poison kernel saw its own LDS stores


def test_fused_refuses_what_it_does_not_cover(torch_cuda):
    """Unaligned audio (a view one sample in) and a 40-filter plan do not
    qualify for the fused kernel: VadError without a workspace, and the
    two-kernel form gives the labels of an aligned copy."""
    torch = torch_cuda
    from vad_amd._lib import VadError
    from vad_amd.config import MfccConfig
    from vad_amd.ffn import FFNClassifier, random_layers
    from vad_amd.pipeline import VadPipeline
    F = 3000
    base = torch.from_numpy(O.synth_clip(O.samples_for_frames(F) + 1, seed=22)).cuda()
    pipe = _pipe(TOPOS[0])
    view = base[1:]  # contiguous, 4-byte but not 8-byte aligned
    assert view.data_ptr() % 8 == 4
    with pytest.raises(VadError):
        pipe.labels(view, fused=True)
    assert torch.equal(pipe.labels(view), pipe.labels(view.clone(), fused=True))
    p40 = VadPipeline(FFNClassifier(random_layers(TOPOS[0], seed=3)), cfg=MfccConfig(n_filters=40))
    assert not p40.fusable
    with pytest.raises(VadError):
        p40.labels(base, fused=True)


def test_fused_out_checks(torch_cuda):
    torch = torch_cuda
    pipe = _pipe(TOPOS[0])
    a = torch.from_numpy(O.synth_clip(O.samples_for_frames(500), seed=23)).cuda()
    with pytest.raises(ValueError):
        pipe.labels(a, out=torch.empty(10, dtype=torch.uint8, device="cuda"))
    with pytest.raises(TypeError):
        pipe.labels(a, out=torch.empty(495, dtype=torch.int32, device="cuda"))
    out = torch.empty(495, dtype=torch.uint8, device="cuda")
    assert pipe.labels(a, out=out) is out
    assert pipe.labels(a, out=out, fused=True) is out
