"""vad_amd -- MI355X-native MFCC + FFN voice-activity detection.

A from-scratch gfx950 implementation of the hot path of nameofuser1/vad:
framing -> 512-point FFT power spectrum -> mel filterbank -> log10 ->
lifter x DCT-II (mfcc.py), the 5-frame feature window
(realtime_analysis/sklearn_analyser.py, dataset/file_processing.py) and the
Keras FFN forward (learning/ffn_trainer.py), behind the reference's own API:
``vad_amd.mfcc`` mirrors ``mfcc.py`` and ``vad_amd.sklearn_analyser``
mirrors ``realtime_analysis/sklearn_analyser.py``.

The arithmetic runs only in HIP kernels (libvad_amd.so, include/vad_amd.h);
importing a compute entry point without the built library raises.
"""
from .config import MfccConfig  # noqa: F401

__version__ = "0.1.0"
