"""Drop-in ``SKLearnAnalyzer`` (reference realtime_analysis/sklearn_analyser.py)
running its per-frame work on the GPU.

Same constructor signature, same ``load_init_inactive_frames`` /
``feed_frame`` behaviour and exceptions:
  * ``ValueError`` when the init-frame count is not 5 (:41-42);
  * ``TypeError`` from ``feed_frame`` when no noise frames were loaded (the
    reference's np.mean([]) -> nan scalar -> len() failure in
    utils.first_order_low_pass, reached from :75 via :122);
  * ``AssertionError('Wrong classifier class')`` for a label other than 0/1 (:82);
  * the returned object is the very frame passed three calls earlier (:76-78).

The noise spectral subtraction (:84-101) has no observable effect (its result
is unused, :122-123), so only its bookkeeping is kept.

Classifier: an ``.npz`` of FFN weights (or a pickled ``FFNClassifier``) runs
the fused GPU step -- MFCC of the new frame, window features and the MFMA FFN
in two kernel launches, state in device memory.  A decision tree (an ``.npz``
node table, or a pickled sklearn ``DecisionTreeClassifier`` -- the classifier
vad.py deploys) is walked on the GPU over the GPU feature row.  Any other
pickled object with ``.predict`` is called with the (1, 39) float64 feature
row computed on the GPU, exactly as the reference calls it.
"""
from __future__ import annotations

import logging
import pickle

import numpy as np
import torch

from . import _lib
from .analyser import Analyser
from .config import FRAMES_BUFFER_SIZE, NOISE_BUFFER_SIZE, PROCESSING_FRAME_INDEX
from .ffn import FFNClassifier
from .mfcc import get_mel_filterbanks
from .plan import MfccPlan, window_features
from .tree import TreeClassifier

logger = logging.getLogger(__name__)


class SKLearnAnalyzer(Analyser):

    FRAMES_BUFFER_SIZE = FRAMES_BUFFER_SIZE
    NOISE_BUFFER_SIZE = NOISE_BUFFER_SIZE
    PROCESSING_FRAME_INDEX = PROCESSING_FRAME_INDEX

    def __init__(self, fname, sample_rate=16000, fft_n=512, mfcc_num=13, low_hz=300, high_hz=8000,
                 fbank_num=26):
        Analyser.__init__(self)
        self.sample_rate = sample_rate
        self.fft_n = fft_n
        self.mfcc_num = mfcc_num
        self.low_hz = low_hz
        self.high_hz = high_hz
        self.fbank_num = fbank_num

        self.filterbank = get_mel_filterbanks(low_hz, high_hz, fft_n, fbank_num, sample_rate)
        self.frames_buffer = []
        self.noise_buffer = []

        if str(fname).endswith(".npz"):
            with np.load(fname, allow_pickle=False) as z:
                is_tree = "threshold" in z.files
            self.classifier = TreeClassifier.load(fname) if is_tree else FFNClassifier.load(fname)
        else:
            # the reference unpickles its classifier file (:34-35); a fitted
            # sklearn decision tree (decision_classifier_trainer.py) moves to
            # the GPU node table, anything else keeps its own predict
            with open(fname, "rb") as f:
                self.classifier = pickle.load(f)
            if TreeClassifier.looks_like_sklearn_tree(self.classifier):
                self.classifier = TreeClassifier.from_sklearn(self.classifier)

        self._plan = MfccPlan(self.filterbank, mfcc_num, fft_n)
        dev = torch.device("cuda", torch.cuda.current_device())
        self._fused = isinstance(self.classifier, FFNClassifier)
        # device state of this stream
        self._ring = torch.zeros((self.FRAMES_BUFFER_SIZE, mfcc_num), dtype=torch.float32, device=dev)
        self._count = torch.zeros((1,), dtype=torch.int32, device=dev)
        self._label = torch.zeros((1,), dtype=torch.uint8, device=dev)
        self._scratch = torch.zeros((1, mfcc_num), dtype=torch.float32, device=dev)
        self._window = torch.zeros((self.FRAMES_BUFFER_SIZE + 1, mfcc_num), dtype=torch.float32,
                                   device=dev)  # foreign-classifier path: window + 1 pad row

    @property
    def frames_mfcc_buffer(self):
        """The MFCC ring in arrival order (host copy, float64) -- introspection only."""
        n = len(self.frames_buffer)
        if self._fused:
            c = int(self._count.item())
            rows = self._ring.cpu().numpy().astype(np.float64)
            return [rows[(c - n + i) % 5] for i in range(n)]
        w = self._window[:self.FRAMES_BUFFER_SIZE].cpu().numpy().astype(np.float64)
        return list(w[self.FRAMES_BUFFER_SIZE - n:])

    def load_init_inactive_frames(self, frames):
        """Noise frames are used for spectral subtraction (:37-44)."""
        if len(frames) != SKLearnAnalyzer.NOISE_BUFFER_SIZE:
            raise ValueError("Number of inactive frame must be the same as BUFFER SIZE")
        self.noise_buffer = [np.asarray(f).astype(np.float32) for f in frames]

    def _frame_to_device(self, frame):
        x = np.ascontiguousarray(np.asarray(frame).astype(np.float32).reshape(-1))
        if x.size == 0:
            raise ValueError("empty frame")
        return torch.from_numpy(x).to(self._ring.device, non_blocking=False)

    def feed_frame(self, frame):
        x = self._frame_to_device(frame)
        if len(self.noise_buffer) == 0:
            # the reference's __noise_spec_subtraction fails on an empty buffer
            raise TypeError("object of type 'numpy.float64' has no len()")
        n = x.numel()
        if self._fused:
            label = self._fused_step(x, n)
        else:
            label = self._foreign_step(x, n)

        if len(self.frames_buffer) < SKLearnAnalyzer.FRAMES_BUFFER_SIZE:
            self.frames_buffer.append(frame)
            return None
        processing_frame = self.frames_buffer[self.PROCESSING_FRAME_INDEX]
        self.frames_buffer.pop(0)
        self.frames_buffer.append(frame)
        if label == 1:
            return processing_frame
        elif label == 0:
            self.noise_buffer.pop(0)
            self.noise_buffer.append(processing_frame)
            return None
        else:
            raise AssertionError('Wrong classifier class')

    def _fused_step(self, x, n):
        ffn = self.classifier.plan
        lib = _lib.lib()
        _lib.check(lib.vad_stream_step(self._plan.handle, ffn.handle, _lib.ptr(x), n, n, 1,
                                       _lib.ptr(self._ring), _lib.ptr(self._count),
                                       _lib.ptr(self._label), _lib.ptr(self._scratch),
                                       _lib.stream_ptr()), "vad_stream_step")
        lab = int(self._label.item())
        return None if lab == 255 else lab

    def _foreign_step(self, x, n):
        label = None
        mf = self._plan.mfcc(x, frame_len=n, frame_stride=n, n=1, out=self._scratch)
        if len(self.frames_buffer) == self.FRAMES_BUFFER_SIZE:
            feats = window_features(self._window, _lib.FEAT_ANALYSER)  # (1, 39)
            if isinstance(self.classifier, TreeClassifier):  # GPU node table
                cls = self.classifier.classes_[int(self.classifier.predict_device(feats).item())]
            else:
                row = feats.cpu().numpy().astype(np.float64).reshape(1, -1)
                cls = self.classifier.predict(row)
            label = 1 if cls == 1 else 0 if cls == 0 else 2
        w = self._window
        w[:self.FRAMES_BUFFER_SIZE - 1].copy_(w[1:self.FRAMES_BUFFER_SIZE].clone())
        w[self.FRAMES_BUFFER_SIZE - 1].copy_(mf[0])
        return label
