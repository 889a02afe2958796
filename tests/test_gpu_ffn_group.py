"""The tile-pair window kernel (ffn_kernel.hip ffn_wave_group_kernel: the
labels-only launches of a 13-64-64-2 analyser network whose layer-1 inputs
the host proved f16-bounded) against the single-tile kernel on the same
MFCC rows: launches that also write the logits (vad_features_ffn_logits)
run ffn_wave_kernel, whose labels come from the same logit difference
(valu_label2), so the two launches' labels must be bit-identical at every
size -- odd tile counts (a wave's second tile clamped and not stored),
single tiles, ragged last tiles, exactly one pair per wave of the full grid
(4,096 waves x 32 windows) and one window past it -- and on windows made
flat (digital silence: NaN features, class 0).  One size is also checked
against the fp64 oracle under the margin rule (test_gpu_parity)."""
import numpy as np
import pytest

from oracle import vad_oracle as O

pytestmark = pytest.mark.gpu

MARGIN_TOL = 0.05
# windows: 1, 15, 16, 17 (one tile, two), 33 (three tiles: odd), 48, 95,
# 4,096 x 32 (one pair per wave of a full grid) and +- 1, 16 x 8,193 + 5
SIZES = [1, 15, 16, 17, 33, 48, 95, 131_071, 131_072, 131_073, 16 * 8_193 + 5]


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    return torch


def mfcc_rows(n_frames, seed):
    """MFCC-like rows (coefficient scales as the pipeline's, c0 ~ -100 .. 50)
    with runs of identical rows (flat windows)."""
    rng = np.random.default_rng(seed)
    scale = np.array([40.0] + [12.0 / (1 + 0.3 * c) for c in range(1, 13)], np.float32)
    m = (rng.standard_normal((n_frames, 13)).astype(np.float32) * scale).astype(np.float32)
    m[:, 0] -= 30.0
    for s in rng.integers(0, max(n_frames - 8, 1), size=max(n_frames // 500, 1)):
        m[s:s + 8] = m[s]  # 8 equal rows: windows entirely inside are flat
    return m


@pytest.mark.parametrize("n_rows", SIZES)
def test_tile_pairs_equal_single_tile(torch_cuda, n_rows):
    from vad_amd import plan as P
    from vad_amd.ffn import TOPOLOGY_BL13, FFNClassifier, random_layers
    torch = torch_cuda
    clf = FFNClassifier(random_layers(TOPOLOGY_BL13, seed=17))
    m = torch.from_numpy(mfcc_rows(n_rows + 5, seed=n_rows)).cuda()
    lab = clf.plan.window_labels(m, P._lib.FEAT_ANALYSER)  # labels only: the tile-pair kernel
    lab_l, logits = P.window_logits(clf.plan, m, P._lib.FEAT_ANALYSER)  # the single-tile kernel
    torch.cuda.synchronize()
    assert lab.shape == (n_rows,)
    np.testing.assert_array_equal(lab.cpu().numpy(), lab_l.cpu().numpy())
    if n_rows == 131_073:
        x = P.window_features(m, P._lib.FEAT_ANALYSER).cpu().numpy()[:, :13].astype(np.float64)
        lay = random_layers(TOPOLOGY_BL13, seed=17)
        flat = np.isnan(x).any(axis=1)
        assert flat.any()
        got = lab.cpu().numpy()
        assert (got[flat] == 0).all()
        ok = ~flat & (O.ffn_margin(np.nan_to_num(x), lay) > MARGIN_TOL)
        np.testing.assert_array_equal(got[ok], O.ffn_labels(np.nan_to_num(x), lay)[ok])
