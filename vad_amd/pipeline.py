"""Clip-level (offline / batch) form of the hot path.

Reference call stack: dataset_creator.py -> Pool.map(
process_file) -> split_into_frames (file_processing.py:80-103) -> per-frame
get_mfcc -> 5-frame feature window (file_processing.py:40-70), with the
analyser's classifier applied to every window (sklearn_analyser.py:52-71).
Here a whole clip resident in HBM is framed, transformed and classified by
two HIP kernels (MFCC rows through a workspace) or one fused kernel (MFCC rows
kept on chip); the host only sizes buffers.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib
from .config import MfccConfig
from .ffn import FFNClassifier
from .plan import MfccPlan, check_out, n_frames, preemphasis, window_features


def split_into_frames(data, frame_size, step, transcription_path=None, frame_rate=None):
    """file_processing.py:80-103 -- list of frame views while len - offset >
    size (with the STM segment gathering of :87-94, see vad_amd.dataset)."""
    from .dataset import split_into_frames as _split
    return _split(data, frame_size, step, transcription_path, frame_rate)


class VadPipeline:
    """MFCC plan + FFN for whole clips on one GPU.

    mode: "analyser" (normalised centre MFCC, sklearn_analyser.py:52-69) or
    "offline" (file_processing.py:40-70 features)."""

    def __init__(self, ffn=None, cfg: MfccConfig = MfccConfig(), mode="analyser"):
        """ffn: an FFNClassifier (or its layers), or a TreeClassifier / fitted
        sklearn DecisionTreeClassifier (the classifier vad.py deploys)."""
        from .tree import TreeClassifier
        self.cfg = cfg
        self.plan = MfccPlan.from_config(cfg)
        if ffn is not None and TreeClassifier.looks_like_sklearn_tree(ffn):
            ffn = TreeClassifier.from_sklearn(ffn)
        if ffn is not None and not isinstance(ffn, (FFNClassifier, TreeClassifier)):
            ffn = FFNClassifier(ffn)
        self.ffn = ffn
        self.mode = _lib.FEAT_ANALYSER if mode == "analyser" else _lib.FEAT_OFFLINE
        self._ws = {}  # (device index, stream) -> workspace

    def n_frames(self, n_samples):
        return n_frames(n_samples, self.cfg.frame_size, self.cfg.hop)

    def _staged(self, audio, stream=None):
        """The clip after the optional pre-emphasis (cfg.preemph; off by default)."""
        if self.cfg.preemph is None:
            return audio
        if audio.dtype != torch.float32:
            audio = audio.float()
        return preemphasis(audio, self.cfg.preemph, stream=stream)

    def mfcc(self, audio, out=None, stream=None):
        """(F, n_mfcc) MFCCs of every frame of a device clip."""
        return self.plan.clip_mfcc(self._staged(audio, stream), self.cfg.frame_size, self.cfg.hop, out=out,
                                   stream=stream)

    def features(self, audio, mode=None, stream=None):
        """(F-5, 3*n_mfcc) feature rows of a device clip."""
        m = self.mfcc(audio, stream=stream)
        return window_features(m, self.mode if mode is None else mode, stream=stream)

    def workspace_bytes(self, n_samples):
        """Device bytes of the two-kernel clip path: the (F, n_mfcc) fp32 MFCC rows."""
        return int(_lib.lib().vad_mfcc_ffn_workspace_bytes(
            self.plan.handle, self.ffn.plan.handle, int(n_samples), self.cfg.frame_size, self.cfg.hop))

    @property
    def fusable(self):
        """The fused kernel (no workspace) applies: reference framing, the
        compiled 26-filter bank, a split-f16 FFN topology."""
        return isinstance(self.ffn, FFNClassifier) and bool(_lib.lib().vad_mfcc_ffn_fusable(
            self.plan.handle, self.ffn.plan.handle, self.cfg.frame_size, self.cfg.hop))

    def _workspace(self, need, device, stream):
        """Cached workspace per (device, stream): a buffer is never shared by
        work on two streams or handed to a kernel on another device."""
        s = stream if stream is not None else torch.cuda.current_stream(device)
        key = (device.index, s.cuda_stream)
        ws = self._ws.get(key)
        if ws is None or ws.numel() < need:
            with torch.cuda.stream(s):
                ws = torch.empty((max(need, 1),), dtype=torch.uint8, device=device)
            self._ws[key] = ws
        return ws

    def labels(self, audio, out=None, stream=None, fused=False):
        """uint8 (F-5,) labels of every window of a device clip; float32
        samples, or int16 PCM as read from a wav file (identical labels).
        fused=False: MFCC kernel + window kernel through a cached workspace
        (the faster form); fused=True: the single fused kernel, MFCC rows kept
        on chip (vad_mfcc_ffn with no workspace) -- identical labels."""
        if self.ffn is None:
            raise ValueError("pipeline has no FFN")
        if not (isinstance(audio, torch.Tensor) and audio.is_cuda
                and audio.dtype in (torch.float32, torch.int16) and audio.is_contiguous()):
            raise TypeError("audio must be a contiguous float32 or int16 CUDA tensor")
        rows = max(self.n_frames(audio.numel()) - 5, 0)
        if out is None:
            out = torch.empty((rows,), dtype=torch.uint8, device=audio.device)
        else:
            check_out(out, (rows,), torch.uint8, audio.device, "out")
        if not isinstance(self.ffn, FFNClassifier):  # decision tree: MFCC, then windows
            if fused:
                raise ValueError("the fused kernel runs the FFN classifiers only")
            return self.ffn.window_labels(self.mfcc(audio, stream=stream), self.mode, out=out,
                                          stream=stream)
        audio = self._staged(audio, stream)
        ws = None if fused else self._workspace(self.workspace_bytes(audio.numel()), audio.device, stream)
        fn = "vad_mfcc_ffn" if audio.dtype == torch.float32 else "vad_mfcc_ffn_i16"
        _lib.check(getattr(_lib.lib(), fn)(
            self.plan.handle, self.ffn.plan.handle, _lib.ptr(audio), audio.numel(),
            self.cfg.frame_size, self.cfg.hop, self.mode, _lib.ptr(out),
            _lib.ptr(ws), 0 if ws is None else ws.numel(), _lib.stream_ptr(stream)), fn)
        return out

    def process_clip(self, data):
        """process_file's feature list for an in-memory clip: (F-5, 3, n_mfcc) float64
        (unnormalised, file_processing.py:40-70)."""
        a = torch.from_numpy(np.ascontiguousarray(np.asarray(data).astype(np.float32))).cuda()
        f = window_features(self.mfcc(a), _lib.FEAT_OFFLINE)
        return f.cpu().numpy().astype(np.float64).reshape(len(f), 3, -1)
