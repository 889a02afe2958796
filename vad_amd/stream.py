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

Host I/O (C5's end-to-end rate includes the copies):
attach_host_io() adds pinned host buffers ``host_inputs`` (K, S, hop) and
``host_labels`` (K, S); step_host() runs one step from the first to the
second -- the H2D copy of every stream's new samples, the hop kernel(s), the
D2H copy of the labels (vad.py:32-59's loop body for S streams at once) --
and capture(host_io=True) records exactly that into the graph, replayed
through vad_graph_launch (hipGraphLaunch, no runtime wrapper in between).

Blocks of hops: with hops_per_step=K a step advances every stream by K hops
(step_block), K x 10 ms of audio per stream, whose new samples sit in the
static input block ``inputs`` (K, S, hop) and whose labels land in
``label_block`` (K, S).  kernel="hop" runs the K hops in ONE launch
(vad_stream_hops: the plan tables staged once, the stream state carried in
registers from hop to hop); capture() records one block into a hipGraph that
reads ``inputs`` in place, so a producer that writes the next block there
(e.g. an H2D copy of the audio devices' buffers) replays with no copy at all.
"""
from __future__ import annotations

import ctypes
import weakref

import torch

from . import _lib
from .config import MfccConfig
from .ffn import FFNClassifier
from .plan import MfccPlan


def hop_rows_disjoint(n_streams, n_hops, block_stride, hop_stride, hop_len):
    """The layouts vad_stream_hops reads in place (capi.hip
    vad_hop_layout_disjoint): one hop only, or hop rows that neither repeat
    nor overlap, in hop-major order ((K, S, hop) blocks) or stream-major
    order (an (S, K * hop) buffer viewed as (K, S, hop))."""
    if n_hops <= 1:
        return True
    if block_stride <= 0:
        return False
    return (block_stride >= (n_streams - 1) * hop_stride + hop_len
            or (block_stride >= hop_len and hop_stride >= (n_hops - 1) * block_stride + hop_len))


class StreamBatch:

    def __init__(self, n_streams, ffn, cfg: MfccConfig = MfccConfig(), device=None, kernel="hop",
                 hops_per_step=1):
        if not isinstance(ffn, FFNClassifier):
            ffn = FFNClassifier(ffn)
        if cfg.preemph is not None:
            raise ValueError("pre-emphasis is a clip-level stage (VadPipeline); streams take raw frames")
        dev = torch.device("cuda", torch.cuda.current_device()) if device is None else device
        if kernel not in ("hop", "three"):
            raise ValueError("kernel must be 'hop' or 'three'")
        if kernel == "hop" and cfg.window is not None:
            raise ValueError("the one-kernel hop has no analysis window; use kernel='three'")
        self.cfg, self.ffn, self.n, self.kernel = cfg, ffn, int(n_streams), kernel
        self.plan = MfccPlan.from_config(cfg)
        S, L, H, C = self.n, cfg.frame_size, cfg.hop, cfg.n_mfcc
        if not 0 < H <= L:
            raise ValueError("hop must be in (0, frame_size]")
        K = int(hops_per_step)
        if K < 1:
            raise ValueError("hops_per_step must be >= 1")
        self.K = K
        self.frames = torch.zeros((S, L), dtype=torch.float32, device=dev)
        # static graph inputs / outputs: K hops of new samples, K label rows
        self.inputs = torch.zeros((K, S, H), dtype=torch.float32, device=dev)
        self.hop_in = self.inputs[0]
        self.ring = torch.zeros((S, 5, C), dtype=torch.float32, device=dev)
        self.count = torch.zeros((S,), dtype=torch.int32, device=dev)
        self.label_block = torch.full((K, S), 255, dtype=torch.uint8, device=dev)
        self.labels = self.label_block[K - 1]
        self.scratch = torch.zeros((S, C), dtype=torch.float32, device=dev)
        self.graph = None
        self.graph_host_io = False
        self.host_inputs = None
        self.host_labels = None

    def prime(self, carry):
        """Set the last frame_size - hop samples of every stream (S, L-H)."""
        L, H = self.cfg.frame_size, self.cfg.hop
        self.frames[:, H:].copy_(carry)

    def reset(self):
        self.frames.zero_()
        self.ring.zero_()
        self.count.zero_()
        self.label_block.fill_(255)

    def _hop_call(self, h, n_hops=1, labels=None):
        """vad_stream_hops with the per-batch arguments prepared once (the
        Python side of a launch is a few microseconds of ctypes marshalling:
        per call only the hop block's address and strides change)."""
        if getattr(self, "_hop_head", None) is None:
            L = self.cfg.frame_size
            self._hop_fn = _lib.lib().vad_stream_hops
            self._hop_head = (self.plan.handle, self.ffn.plan.handle, _lib.ptr(self.frames), L, L)
            self._hop_mid = (_lib.ptr(self.ring), _lib.ptr(self.count))
            self._hop_labels = {}
        lab = self.labels if labels is None else labels
        key = (lab.data_ptr(), n_hops)
        tail = self._hop_labels.get(key)
        if tail is None:
            tail = (ctypes.c_void_p(lab.data_ptr()), lab.stride(0) if lab.dim() == 2 else 0)
            self._hop_labels[key] = tail
        rc = self._hop_fn(*self._hop_head, ctypes.c_void_p(h.data_ptr()), h.stride(-2), self.cfg.hop, self.n,
                          n_hops, h.stride(0) if h.dim() == 3 else 0, *self._hop_mid, *tail,
                          _lib.stream_ptr())
        if rc:
            _lib.check(rc, "vad_stream_hops")

    def _three(self, h, labels):
        L, H = self.cfg.frame_size, self.cfg.hop
        lib = _lib.lib()
        _lib.check(lib.vad_stream_push_hop(_lib.ptr(self.frames), L, L, ctypes.c_void_p(h.data_ptr()), h.stride(0),
                                           H, self.n, _lib.stream_ptr()), "vad_stream_push_hop")
        _lib.check(lib.vad_stream_step(
            self.plan.handle, self.ffn.plan.handle, _lib.ptr(self.frames), L, L, self.n,
            _lib.ptr(self.ring), _lib.ptr(self.count), ctypes.c_void_p(labels.data_ptr()),
            _lib.ptr(self.scratch), _lib.stream_ptr()), "vad_stream_step")

    def _body(self, hop=None):
        """One hop (K = 1) from `hop` or the static input."""
        h = self.hop_in if hop is None else hop
        if self.kernel == "hop":
            self._hop_call(h)
        else:
            self._three(h, self.labels)

    def _block_body(self):
        """K hops from the static input block into label_block."""
        if self.kernel == "hop":
            self._hop_call(self.inputs, self.K, self.label_block)
        else:
            for k in range(self.K):
                self._three(self.inputs[k], self.label_block[k])

    def step(self, new_samples=None):
        """Advance every stream by one hop (new_samples: (S, hop) device fp32;
        None: the hop already written into ``hop_in``).  hops_per_step == 1."""
        if self.K != 1:
            raise ValueError("this batch advances hops_per_step hops at a time: use step_block")
        if new_samples is not None and (new_samples.shape != self.hop_in.shape
                                        or new_samples.dtype != torch.float32 or not new_samples.is_cuda):
            raise ValueError(f"new_samples must be a CUDA float32 tensor of shape {tuple(self.hop_in.shape)}")
        if self.graph is not None and not self.graph_host_io:
            if new_samples is not None:
                self.hop_in.copy_(new_samples)
            self._replay()
        elif self.kernel == "hop" and new_samples is not None and new_samples.stride(1) == 1:
            self._body(new_samples)  # read in place: no copy
        else:
            if new_samples is not None:
                self.hop_in.copy_(new_samples)
            self._body()
        return self.labels

    def step_block(self, new_samples=None):
        """Advance every stream by K = hops_per_step hops; new_samples: (K, S,
        hop) device fp32, or None when the block was written into ``inputs``
        (the graph's static input: no copy).  Returns label_block (K, S)."""
        if new_samples is not None:
            if new_samples.shape != self.inputs.shape or new_samples.dtype != torch.float32 \
                    or not new_samples.is_cuda:
                raise ValueError(f"new_samples must be a CUDA float32 tensor of shape {tuple(self.inputs.shape)}")
            if (self.graph is None or self.graph_host_io) and self.kernel == "hop" and new_samples.stride(2) == 1 \
                    and hop_rows_disjoint(self.n, self.K, new_samples.stride(0), new_samples.stride(1), self.cfg.hop):
                self._hop_call(new_samples, self.K, self.label_block)  # read in place
                return self.label_block
            self.inputs.copy_(new_samples)
        if self.graph is not None and not self.graph_host_io:
            self._replay()
        else:
            self._block_body()
        return self.label_block

    def attach_host_io(self):
        """Pinned host buffers for step_host: host_inputs (K, S, hop) fp32,
        host_labels (K, S) uint8."""
        if self.host_inputs is None:
            self.host_inputs = torch.zeros(tuple(self.inputs.shape), dtype=torch.float32, pin_memory=True)
            self.host_labels = torch.full(tuple(self.label_block.shape), 255, dtype=torch.uint8,
                                          pin_memory=True)
        return self.host_inputs, self.host_labels

    def _host_body(self):
        self.inputs.copy_(self.host_inputs, non_blocking=True)
        if self.K == 1:
            self._body()
        else:
            self._block_body()
        self.host_labels.copy_(self.label_block, non_blocking=True)

    def _replay(self):
        _lib.check(self._graph_launch(self._graph_plan, _lib.stream_ptr()), "vad_graph_plan_launch")

    def step_host(self):
        """One step (K hops) from ``host_inputs`` to ``host_labels``: H2D
        copy, the hop kernel(s), D2H copy, all on the current stream (the
        caller synchronises it before reading host_labels).  Replays the
        graph when capture(host_io=True) recorded one.  The copies are
        asynchronous: a producer rewrites host_inputs only once the stream
        has passed the previous step's H2D copy (a stream or event sync, as
        vad.py's loop would do before reading the labels anyway)."""
        if self.host_inputs is None:
            raise ValueError("attach_host_io() (or capture(host_io=True)) first")
        if self.graph is not None and self.graph_host_io:
            self._replay()
        else:
            self._host_body()
        return self.host_labels

    def capture(self, host_io=False):
        """Capture one step (K hops) into a hipGraph (torch.cuda.CUDAGraph);
        step() / step_block() replay it, reading the static ``inputs``.  With
        host_io the graph also holds the H2D copy from ``host_inputs`` and the
        D2H copy to ``host_labels`` (replayed by step_host)."""
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        saved = (self.frames.clone(), self.ring.clone(), self.count.clone(), self.label_block.clone())
        if host_io:
            self.attach_host_io()
            body = self._host_body
        else:
            body = self._body if self.K == 1 else self._block_body
        with torch.cuda.stream(s):
            body()  # warm-up (first launch sets kernel attributes)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        self.frames.copy_(saved[0]); self.ring.copy_(saved[1])
        self.count.copy_(saved[2]); self.label_block.copy_(saved[3])
        # keep_graph: the captured hipGraph_t stays alive beside its exec, so
        # the replay plan can read its nodes (vad_graph_plan_create: a
        # one-kernel-node graph -- the one-hop step -- is dispatched as its
        # node, whose host cost is a launch's, not hipGraphLaunch's)
        g = torch.cuda.CUDAGraph(keep_graph=True)
        with torch.cuda.graph(g):
            body()
        g.instantiate()
        self._drop_graph_plan()
        lib = _lib.lib()
        h = ctypes.c_void_p()
        _lib.check(lib.vad_graph_plan_create(ctypes.c_void_p(g.raw_cuda_graph()),
                                             ctypes.c_void_p(g.raw_cuda_graph_exec()), ctypes.byref(h)),
                   "vad_graph_plan_create")
        self._graph_plan = h
        self._graph_launch = lib.vad_graph_plan_launch
        self._graph_plan_free = weakref.finalize(self, lib.vad_graph_plan_destroy, h)
        self.graph = g
        self.graph_host_io = bool(host_io)
        return g

    @property
    def graph_direct(self):
        """True when replays dispatch the captured graph's single kernel node."""
        return self.graph is not None and bool(_lib.lib().vad_graph_plan_direct(self._graph_plan))

    def _drop_graph_plan(self):
        fin = getattr(self, "_graph_plan_free", None)
        if fin is not None:
            fin()  # the plan before the graph it points into
        self._graph_plan = None
