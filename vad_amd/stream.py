"""Many concurrent analyser streams on one GPU (BASELINE config 5).

Each of S streams behaves like its own ``SKLearnAnalyzer.feed_frame`` loop
(realtime_analysis/sklearn_analyser.py:46-82) fed with the 400-sample frame
that ends at the newest sample, advanced one hop (160 samples = 10 ms) per
step.  One step = three HIP kernels -- frame assembly (shift by one hop,
append the new samples, in place), MFCC, window features + FFN -- replayable
as one hipGraph.

labels[s] after a step is the class of stream s's window centred three steps
earlier, or 255 during each stream's first five steps (feed_frame returns
None for its first five calls, :48-50).
"""
from __future__ import annotations

import torch

from . import _lib
from .config import MfccConfig
from .ffn import FFNClassifier
from .plan import MfccPlan


class StreamBatch:

    def __init__(self, n_streams, ffn, cfg: MfccConfig = MfccConfig(), device=None):
        if not isinstance(ffn, FFNClassifier):
            ffn = FFNClassifier(ffn)
        if cfg.preemph is not None:
            raise ValueError("pre-emphasis is a clip-level stage (VadPipeline); streams take raw frames")
        dev = torch.device("cuda", torch.cuda.current_device()) if device is None else device
        self.cfg, self.ffn, self.n = cfg, ffn, int(n_streams)
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

    def _body(self):
        L, H = self.cfg.frame_size, self.cfg.hop
        lib = _lib.lib()
        _lib.check(lib.vad_stream_push_hop(_lib.ptr(self.frames), L, L, _lib.ptr(self.hop_in), H, H,
                                           self.n, _lib.stream_ptr()), "vad_stream_push_hop")
        _lib.check(lib.vad_stream_step(
            self.plan.handle, self.ffn.plan.handle, _lib.ptr(self.frames), L, L, self.n,
            _lib.ptr(self.ring), _lib.ptr(self.count), _lib.ptr(self.labels),
            _lib.ptr(self.scratch), _lib.stream_ptr()), "vad_stream_step")

    def step(self, new_samples=None):
        """Advance every stream by one hop (new_samples: (S, hop) device fp32)."""
        if new_samples is not None:
            self.hop_in.copy_(new_samples)
        if self.graph is not None:
            self.graph.replay()
        else:
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
