"""SimpleAnalyser (realtime_analysis/simple_analyzer.py) against the trace of
the unmodified reference class (tests/golden/simple.npz, made by
tests/golden/gen_simple.py with pyAudioAnalysis's stEnergy / stZCR restated).

CPU tests drive vad_amd's state machine with the oracle's per-frame
features; GPU tests use the fp64 HIP features (vad_simple_features)."""
import numpy as np
import pytest

from oracle import vad_oracle as O
from vad_amd.simple_analyser import SimpleAnalyser

CASES = ["a", "b", "c"]


def _oracle_features(self, frames):
    rows = np.asarray(frames, np.float64).reshape(-1, self.frame_size)
    return np.array([O.simple_frame_features(r, self.frame_size, self.frame_rate) for r in rows])


def _run(sa, g, case, batch=False):
    fs, nb = int(g[f"{case}_meta"][0]), int(g[f"{case}_meta"][1])
    frames = list(g[f"{case}_frames"])
    sa.load_init_inactive_frames(frames[:nb])
    rec = []
    if batch:
        rets = sa.classify_frames(frames[nb:])
        return np.array(rets, float)
    for fr in frames[nb:]:
        r = sa.feed_frame(fr)
        rec.append([float(r), float(sa.silence), sa.energy_thresh, sa.spectral_std_thresh]
                   + list(sa.spectral_energy_bands_thresh))
    return np.asarray(rec)


@pytest.mark.parametrize("case", CASES)
def test_state_machine_matches_reference(golden, monkeypatch, case):
    g = golden("simple")
    monkeypatch.setattr(SimpleAnalyser, "frame_features", _oracle_features)
    fs, nb, fftn, pad, fb = map(int, g[f"{case}_meta"])
    sa = SimpleAnalyser(16000, fs, nb)
    assert (sa.fftn, sa.fft_extended_zeros, sa.fftn_for_band) == (fftn, pad, fb)
    tr = _run(sa, g, case)
    ref = g[f"{case}_trace"]
    assert np.array_equal(tr[:, :2], ref[:, :2])
    assert np.allclose(tr[:, 2:], ref[:, 2:], rtol=1e-12, atol=0)


def test_exceptions(golden, monkeypatch):
    g = golden("simple")
    monkeypatch.setattr(SimpleAnalyser, "frame_features", _oracle_features)
    sa = SimpleAnalyser(16000, 400, 5)
    with pytest.raises(Exception, match="not initialized"):
        sa.feed_frame(np.zeros(400))
    with pytest.raises(Exception, match="Expected 5 initial frames"):
        sa.load_init_inactive_frames([np.zeros(400)] * 4)
    sa.load_init_inactive_frames(list(g["a_frames"][:5]))
    with pytest.raises(Exception, match="Wrong frame size"):
        sa.feed_frame(np.zeros(399))


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES)
def test_gpu_features_match_oracle(golden, case):
    g = golden("simple")
    fs, nb = int(g[f"{case}_meta"][0]), int(g[f"{case}_meta"][1])
    sa = SimpleAnalyser(16000, fs, nb)
    frames = g[f"{case}_frames"]
    got = sa.frame_features(frames)
    ref = np.array([O.simple_frame_features(r, fs, 16000) for r in frames])
    assert np.array_equal(got[:, 0], ref[:, 0])   # sum of squares of integers: exact
    assert np.array_equal(got[:, 1], ref[:, 1])   # crossing counts: exact
    assert np.allclose(got[:, 2:], ref[:, 2:], rtol=1e-11, atol=0)


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES)
def test_gpu_trace_matches_reference(golden, case):
    g = golden("simple")
    fs, nb = int(g[f"{case}_meta"][0]), int(g[f"{case}_meta"][1])
    tr = _run(SimpleAnalyser(16000, fs, nb), g, case)
    ref = g[f"{case}_trace"]
    assert np.array_equal(tr[:, :2], ref[:, :2])
    assert np.allclose(tr[:, 2:], ref[:, 2:], rtol=1e-10, atol=0)
    batch = _run(SimpleAnalyser(16000, fs, nb), g, case, batch=True)
    assert np.array_equal(batch, ref[:, 0])
