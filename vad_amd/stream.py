"""Many concurrent analyser streams on one GPU (BASELINE config 5).

Each of S streams behaves like its own ``SKLearnAnalyzer.feed_frame`` loop
(realtime_analysis/sklearn_analyser.py:46-82) fed with the 400-sample frame
that ends at the newest sample, advanced one hop (160 samples = 10 ms) per
step.  Two forms of a step, identical semantics:
  kernel="hop"    ONE HIP kernel, one wave per stream (vad_stream_hop): frame
                  assembly, FFT, mel / log / DCT, window features, FFN (exact
                  f32 on the VALU) -- latency first;
  kernel="three"  frame assembly (shift by one hop, append the new samples,
                  in place), the clip MFCC kernel, the window features + MFMA
                  FFN kernel -- three launches, replayable as one hipGraph.

labels[s] after a step is the class of stream s's window centred three steps
earlier, or 255 during each stream's first five steps (feed_frame returns
None for its first five calls, :48-50).
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from .config import MfccConfig
from .ffn import FFNClassifier
from .plan import MfccPlan


class StreamBatch:

    def __init__(self, n_streams, ffn, cfg: MfccConfig = MfccConfig(), device=None, kernel="hop"):
        if not isinstance(ffn, FFNClassifier):
            ffn = FFNClassifier(ffn)
        if cfg.preemph is not None:
            raise ValueError("pre-emphasis is a clip-level stage (VadPipeline); streams take raw frames")
        dev = torch.device("cuda", torch.cuda.current_device()) if device is None else device
        if kernel not in ("hop", "three"):
            raise ValueError("kernel must be 'hop' or 'three'")
        self.cfg, self.ffn, self.n, self.kernel = cfg, ffn, int(n_streams), kernel
        self.plan = MfccPlan.from_config(cfg)
        S, L, H, C = self.n, cfg.frame_size, cfg.hop, cfg.n_mfcc
        if not 0 < H <= L:
            raise ValueError("hop must be in (0, frame_size]")
        self.frames = torch.zeros((S, L), dtype=torch.float32, device=dev)
        self.hop_in = torch.zeros((S, H), dtype=torch.float32, device=dev)   # static graph input
        self.ring = torch.zeros((S, 5, C), dtype=torch.float32, device=dev)
        self.count = torch.zeros((S,), dtype=torch.int32, device=dev)
        self.labels = torch.full((S,), 255, dtype=torch.uint8, device=dev)
        self.scratch = torch.zeros((S, C), dtype=torch.float32, device=dev)
        self.graph = None

    def prime(self, carry):
        """Set the last frame_size - hop samples of every stream (S, L-H)."""
        L, H = self.cfg.frame_size, self.cfg.hop
        self.frames[:, H:].copy_(carry)

    def reset(self):
        self.frames.zero_()
        self.ring.zero_()
        self.count.zero_()
        self.labels.fill_(255)

    def _hop_call(self, h):
        """vad_stream_hop with the per-batch arguments prepared once (the
        Python side of a hop is a few microseconds of ctypes marshalling)."""
        if getattr(self, "_hop_args", None) is None:
            L, H = self.cfg.frame_size, self.cfg.hop
            self._hop_fn = _lib.lib().vad_stream_hop
            self._hop_args = (self.plan.handle, self.ffn.plan.handle, _lib.ptr(self.frames), L, L)
            self._hop_tail = (H, self.n, _lib.ptr(self.ring), _lib.ptr(self.count), _lib.ptr(self.labels))
        rc = self._hop_fn(*self._hop_args, ctypes.c_void_p(h.data_ptr()), h.stride(0), *self._hop_tail,
                          _lib.stream_ptr())
        if rc:
            _lib.check(rc, "vad_stream_hop")

    def _body(self, hop=None):
        L, H = self.cfg.frame_size, self.cfg.hop
        lib = _lib.lib()
        if self.kernel == "hop":
            self._hop_call(self.hop_in if hop is None else hop)
            return
        _lib.check(lib.vad_stream_push_hop(_lib.ptr(self.frames), L, L, _lib.ptr(self.hop_in), H, H,
                                           self.n, _lib.stream_ptr()), "vad_stream_push_hop")
        _lib.check(lib.vad_stream_step(
            self.plan.handle, self.ffn.plan.handle, _lib.ptr(self.frames), L, L, self.n,
            _lib.ptr(self.ring), _lib.ptr(self.count), _lib.ptr(self.labels),
            _lib.ptr(self.scratch), _lib.stream_ptr()), "vad_stream_step")

    def step(self, new_samples=None):
        """Advance every stream by one hop (new_samples: (S, hop) device fp32)."""
        if new_samples is not None and (new_samples.shape != self.hop_in.shape
                                        or new_samples.dtype != torch.float32 or not new_samples.is_cuda):
            raise ValueError(f"new_samples must be a CUDA float32 tensor of shape {tuple(self.hop_in.shape)}")
        if self.graph is not None:
            if new_samples is not None:
                self.hop_in.copy_(new_samples)
            self.graph.replay()
        elif self.kernel == "hop" and new_samples is not None and new_samples.stride(1) == 1:
            self._body(new_samples)  # read in place: no copy
        else:
            if new_samples is not None:
                self.hop_in.copy_(new_samples)
            self._body()
        return self.labels

    def capture(self):
        """Capture one step into a hipGraph (torch.cuda.CUDAGraph); step() replays it."""
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        saved = (self.frames.clone(), self.ring.clone(), self.count.clone(), self.labels.clone())
        with torch.cuda.stream(s):
            self._body()  # warm-up (first launch sets kernel attributes)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        self.frames.copy_(saved[0]); self.ring.copy_(saved[1])
        self.count.copy_(saved[2]); self.labels.copy_(saved[3])
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self._body()
        self.graph = g
        return g
