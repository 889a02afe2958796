"""SimpleAnalyser fixture (tests/golden/simple.npz): the UNMODIFIED reference
class (realtime_analysis/simple_analyzer.py) driven over a synthetic stream.

pyAudioAnalysis (its stEnergy / stZCR) is absent here; a stub module with
the published definitions (oracle.vad_oracle.st_energy / st_zcr) stands in.
``frame_size`` is an int whose arithmetic keeps Py2 integer division
(simple_analyzer.py:227 ``(val - frame_size) / 2``).  The class logs every
frame to realtime.log / frames.log in the working directory, so it runs in a
temporary one.  Recorded per feed_frame call: the return value, the silence
flag and the three thresholds after the call.

    python tests/golden/gen_simple.py
"""
import os
import sys
import tempfile
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from oracle import vad_oracle as O  # noqa: E402


class Py2Int(int):
    def __sub__(self, o):
        return Py2Int(int(self) - int(o))

    def __rsub__(self, o):
        return Py2Int(int(o) - int(self))

    def __truediv__(self, o):
        return Py2Int(int(self) // int(o))


def stream_frames(n, frame_size, seed, n_noise):
    """n_noise quiet frames, then noise (sigma 5) with voiced bursts (150-250
    Hz, harmonics falling as 1/h^2) and loud noise bursts; int-valued float64."""
    rng = np.random.default_rng(seed)
    t = np.arange(frame_size)
    out = []
    state, amp, left = "quiet", 1.0, 0
    for i in range(n):
        if i >= n_noise and left <= 0:
            state = rng.choice(["quiet", "voiced", "loud"], p=[0.45, 0.45, 0.10])
            left = int(rng.integers(3, 40))
            amp = 10 ** rng.uniform(2.0, 3.7)
        left -= 1
        x = rng.normal(0, 5, frame_size)
        if state == "voiced":
            f0 = rng.uniform(150, 250)
            for h in range(1, 21):
                x += amp / h ** 2 * np.sin(2 * np.pi * f0 * h * (t + i * frame_size) / 16000
                                           + rng.uniform(0, 0.3))
        elif state == "loud":
            x += rng.normal(0, amp / 4, frame_size)
        out.append(np.rint(x))
    return out


def main():
    aud = types.ModuleType("pyAudioAnalysis.audioFeatureExtraction")
    aud.stEnergy, aud.stZCR = O.st_energy, O.st_zcr
    pkg = types.ModuleType("pyAudioAnalysis")
    pkg.audioFeatureExtraction = aud
    sys.modules["pyAudioAnalysis"] = pkg
    sys.modules["pyAudioAnalysis.audioFeatureExtraction"] = aud
    sys.path.insert(0, os.path.join(REF, "realtime_analysis"))
    cwd = os.getcwd()
    os.chdir(tempfile.mkdtemp())
    try:
        import simple_analyzer
        out = {}
        for case, (fs, nb, seed, n) in {"a": (400, 5, 3, 600), "b": (512, 3, 4, 300), "c": (401, 4, 5, 200)}.items():
            sa = simple_analyzer.SimpleAnalyser(16000, Py2Int(fs), nb)
            frames = stream_frames(nb + n, fs, seed, nb)
            sa.load_init_inactive_frames(frames[:nb])
            rec = []
            for fr in frames[nb:]:
                r = sa.feed_frame(fr)
                rec.append([float(r), float(sa.silence), sa.energy_thresh, sa.spectral_std_thresh]
                           + list(sa.spectral_energy_bands_thresh))
            out[f"{case}_frames"] = np.asarray(frames)
            out[f"{case}_trace"] = np.asarray(rec)
            out[f"{case}_meta"] = np.array([fs, nb, sa.fftn, sa.fft_extended_zeros, sa.fftn_for_band])
            sa.de_init()
        np.savez_compressed(os.path.join(HERE, "simple.npz"), **out)
        for c in ("a", "b", "c"):
            tr = out[f"{c}_trace"]
            print(c, "active share", tr[:, 0].mean(), "silence share", tr[:, 1].mean(),
                  out[f"{c}_meta"])
    finally:
        os.chdir(cwd)


if __name__ == "__main__":
    main()
