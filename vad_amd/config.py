"""Constants and the MFCC configuration (reference config.py:20-27, labels
config.py:45-47, analyser defaults realtime_analysis/sklearn_analyser.py:21)."""
from __future__ import annotations

from dataclasses import dataclass

SAMPLERATE = 16000
FRAME_SIZE = 400
FRAME_STEP = 160
LOW_HZ = 300
HIGH_HZ = 8000
FILTERBANKS_NUM = 26
MFCC_NUM = 13
FFT_N = 512

NONE_VOICED = 0
VOICED = 1
MUSIC = 2

FRAMES_BUFFER_SIZE = 5       # sklearn_analyser.py:17
NOISE_BUFFER_SIZE = 5        # sklearn_analyser.py:18
PROCESSING_FRAME_INDEX = 2   # sklearn_analyser.py:19


@dataclass(frozen=True)
class MfccConfig:
    """One MFCC configuration.

    preemph / window are optional stages BASELINE's north_star names that the
    reference pipeline does NOT have (mfcc.py:59-61 feeds raw frames to the
    FFT): default off, and with both off every output is bit-identical to the
    reference-parity path.  preemph = a runs y[t] = x[t] - a x[t-1] over the
    clip before framing; window = "hamming" multiplies each frame by
    numpy.hamming(frame_size) before the FFT (python_speech_features
    conventions; parity pinned to the oracle's restatement only)."""

    sample_rate: int = SAMPLERATE
    frame_size: int = FRAME_SIZE
    hop: int = FRAME_STEP
    fft_n: int = FFT_N
    n_filters: int = FILTERBANKS_NUM
    n_mfcc: int = MFCC_NUM
    low_hz: float = LOW_HZ
    high_hz: float = HIGH_HZ
    lifter: int = 22   # mfcc.py:85 default, used by every reference call
    preemph: float | None = None   # off: not in the reference
    window: str | None = None      # None (rectangular, the reference) or "hamming"
