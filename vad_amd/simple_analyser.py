"""Drop-in ``SimpleAnalyser`` (reference realtime_analysis/simple_analyzer.py):
the energy / zero-crossing / spectral voice-activity detector, the second
``Analyser`` implementation.

The per-frame measurements -- stEnergy, stZCR, the magnitude spectrum's
std and its four 1-kHz band energies (pyAudioAnalysis stEnergy / stZCR
semantics) -- run on the GPU in fp64 (``vad_simple_features``).  Everything
the reference recomputes from its noise buffer on every update is a function
of those per-frame values, so the noise buffer keeps each noise frame's
features; the thresholds, the 20-frame status buffer and the silence state
are the reference's, update for update.  ``classify_frames`` runs a whole
sequence of frames with one kernel launch and the same state machine.

Same constructor, methods and exceptions as the reference (``Exception``
for an uninitialised analyser, a wrong frame size or a wrong init-frame
count).  Frames are read as fp32 samples (exact for int16 audio); the
reference's own arithmetic on int16 / float32 frames (int16 overflow in
``frame ** 2``, float32 sums) is not reproduced: features are the float64
values the reference computes for float64 frames.  Logging is lazy and goes
to the module logger (the reference writes realtime.log / frames.log).
"""
from __future__ import annotations

import logging

import numpy as np
import torch

from . import _lib
from .analyser import Analyser

logger = logging.getLogger(__name__)


class SimpleAnalyser(Analyser):

    TEMP_BUFFER_SIZE = 20
    TEMP_ACTIVE_THRESHOLD = 5
    TEMP_INACTIVE_THRESHOLD = 15

    def __init__(self, frame_rate, frame_size, noise_buf_len):
        Analyser.__init__(self)
        self.frame_rate = frame_rate
        self.frame_size = int(frame_size)
        self.spectral_bands = 4
        self.spectral_bin_width = 0
        self.noise_buf_len = int(noise_buf_len)
        self.silence = True
        self.temp_buffer = [False] * self.TEMP_BUFFER_SIZE
        self.logger = logger
        self.frame_number = 0
        self.fft_extended_zeros = 0
        self.fftn = 0
        self.fftn_for_band = 0
        self.noise_pointer = 0
        # features of the noise-buffer frames: [energy, zcr, std, bands...]
        self._noise_feats = np.zeros((self.noise_buf_len, 3 + self.spectral_bands), np.float64)
        self.energy_thresh = 0.0
        self.energy_std = 0.0
        self.energy_k = 2.0
        self.spectral_std_thresh = 0.0
        self.spectal_std_k = 2.0
        self.spectral_energy_bands_thresh = np.zeros((self.spectral_bands,), np.float64)
        self.spectral_energy_bands_k = 3.0
        self._choose_optimal_fft_size()
        self.initialized = False
        self.inactive_in_row = 5
        self.active_in_row = 0

    def de_init(self):
        """The reference closes its log files (:66-73); nothing to release here."""

    # -- GPU features ---------------------------------------------------------
    def _choose_optimal_fft_size(self):
        """:221-236 (Py2 integer division)."""
        val = 2
        while val < self.frame_size:
            val <<= 1
        self.fftn = val
        self.fft_extended_zeros = (val - self.frame_size) // 2 + (val - self.frame_size) % 2
        self.spectral_bin_width = (self.frame_rate + 0.0) / (self.fftn + 0.0)
        self.fftn_for_band = int(1000 / self.spectral_bin_width)
        if self.fftn < self.spectral_bands * self.fftn_for_band:
            raise Exception("Can't get spectral bands. FFTN is small")

    def _fft_len(self):
        return self.frame_size + 2 * self.fft_extended_zeros

    def frame_features(self, frames):
        """(n, 7) float64 [stEnergy, stZCR*frame_size, std|fft|, 4 band energies]
        of n frames (rows of a 2-D array or a list of equal-length frames)."""
        x = np.ascontiguousarray(np.asarray(frames, np.float32).reshape(-1, self.frame_size))
        n = x.shape[0]
        k = 3 + self.spectral_bands
        if n == 0:
            return np.zeros((0, k))
        t = torch.from_numpy(x).cuda()
        out = torch.empty((n, k), dtype=torch.float64, device=t.device)
        _lib.check(_lib.lib().vad_simple_features(
            _lib.ptr(t), n, self.frame_size, self.frame_size, self._fft_len(),
            self.fft_extended_zeros, self.fftn_for_band, self.spectral_bands, _lib.ptr(out),
            _lib.stream_ptr()), "vad_simple_features")
        return out.cpu().numpy()

    # -- reference API ----------------------------------------------------------
    def load_init_inactive_frames(self, frames):
        """:115-135."""
        if len(frames) != self.noise_buf_len:
            raise Exception("Expected " + str(self.noise_buf_len) + " initial frames. Got "
                            + str(len(frames)))
        rows = [np.asarray(f, np.float64).reshape(-1)[:self.frame_size] for f in frames]
        self._noise_feats[:] = self.frame_features(np.asarray(rows))
        self.energy_thresh = self._inactive_mean_st_energy()
        self.spectral_energy_bands_thresh = self._inactive_spectral_energy_mean_bands()
        self.spectral_std_thresh = self._inactive_mean_spectral_std()
        self.logger.debug("Init thresholds: energy %s, bands %s, spectral std %s",
                          self.energy_thresh, self.spectral_energy_bands_thresh,
                          self.spectral_std_thresh)
        self.initialized = True

    def feed_frame(self, frame):
        """:79-113: True (active) / False (inactive)."""
        if not self.initialized:
            raise Exception("Analyser not initialized")
        if len(frame) != self.frame_size:
            raise Exception("Wrong frame size. Expected " + str(self.frame_size) + " bytes. Got "
                            + str(len(frame)))
        return self._step(self.frame_features(np.asarray(frame)[None, :])[0])

    def classify_frames(self, frames):
        """feed_frame over a sequence of frames (one kernel launch for all
        their features); returns the list of booleans feed_frame would."""
        if not self.initialized:
            raise Exception("Analyser not initialized")
        frames = list(frames)
        for fr in frames:
            if len(fr) != self.frame_size:
                raise Exception("Wrong frame size. Expected " + str(self.frame_size)
                                + " bytes. Got " + str(len(fr)))
        feats = self.frame_features(np.asarray(frames)) if frames else []
        return [self._step(f) for f in feats]

    # -- the reference's state machine on per-frame features --------------------
    def _step(self, f):
        self.frame_number += 1
        status = self._classify(f)
        self._add_status_to_temp_buffer(status)
        active, inactive = self._get_temp_buffer_statuses()
        self.logger.debug("Frame %d: %s", self.frame_number, "ACTIVE" if status else "INACTIVE")
        if status:
            if self.silence and active >= self.TEMP_ACTIVE_THRESHOLD:
                self.silence = False
            return True
        if self.silence:
            self._add_inactive_frame(f)
            return False
        if inactive >= self.TEMP_INACTIVE_THRESHOLD:
            self._add_inactive_frame(f)
            self.silence = True
        return True

    def _classify(self, f):
        """:140-160."""
        if self._is_spectral_energy_active(f) and self._is_zrc_active(f):
            return True
        if self._is_zrc_active(f) and self._is_energy_active(f) and self._is_spectral_std_active(f):
            return True
        return False

    def _is_energy_active(self, f):
        return f[0] > self.energy_k * self.energy_thresh

    def _is_spectral_energy_active(self, f):
        """:174-197: band 0-1 kHz and two of the others above k x threshold."""
        b, th, k = f[3:], self.spectral_energy_bands_thresh, self.spectral_energy_bands_k
        if b[0] > th[0] * k:
            return sum(1 for i in range(1, self.spectral_bands) if b[i] > th[i] * k) >= 2
        return False

    def _is_spectral_std_active(self, f):
        return f[2] > self.spectral_std_thresh * self.spectal_std_k

    @staticmethod
    def _is_zrc_active(f):
        return 20 >= f[1] >= 5

    def _add_inactive_frame(self, f):
        """:244-255: the frame's features replace the oldest noise entry."""
        self._noise_feats[self.noise_pointer] = f
        self._update_energy_threshold()
        self._update_spectral_energy_bands_threshold()
        self._update_spectral_std_threshold()
        self.noise_pointer = 0 if self.noise_pointer == self.noise_buf_len - 1 else self.noise_pointer + 1

    def _update_spectral_std_threshold(self):
        p = 0.25
        self.spectral_std_thresh = (1 - p) * self.spectral_std_thresh + p * self._inactive_mean_spectral_std()

    def _inactive_mean_spectral_std(self):
        return np.mean(self._noise_feats[:, 2])

    def _update_energy_threshold(self):
        p = 0.25
        self.energy_thresh = (1 - p) * self.energy_thresh + p * self._inactive_mean_st_energy()

    def _inactive_mean_st_energy(self):
        # the reference stores the energies in a uint32 array (:292-299):
        # truncation toward zero
        return np.mean(self._noise_feats[:, 0].astype(np.uint32))

    def _update_spectral_energy_bands_threshold(self):
        p = 0.25
        new = self._inactive_spectral_energy_mean_bands()
        for i in range(self.spectral_bands):
            self.spectral_energy_bands_thresh[i] = (1 - p) * self.spectral_energy_bands_thresh[i] + p * new[i]

    def _inactive_spectral_energy_mean_bands(self):
        return np.mean(self._noise_feats[:, 3:], axis=0)

    @staticmethod
    def get_new_p(sigma_new, sigma_old):
        """:402-415 (unused by the reference's updates)."""
        y = sigma_new / sigma_old
        if y >= 1.25:
            return 0.25
        if 1.25 >= y >= 1.10:
            return 0.20
        if 1.10 >= y >= 1.0:
            return 0.15
        if 1.0 >= y:
            return 0.10

    def _get_temp_buffer_statuses(self):
        active = sum(1 for s in self.temp_buffer if s)
        return active, len(self.temp_buffer) - active

    def _add_status_to_temp_buffer(self, status):
        if len(self.temp_buffer) == self.TEMP_BUFFER_SIZE:
            self.temp_buffer.pop(0)
        self.temp_buffer.append(status)
