"""Multi-GPU clip sharding (BASELINE config 4).

Independent clips shard across ranks with no data-path collective: rank r
classifies its own clips on its own GPU.  One long clip splits at frame
boundaries with a halo: rank r's windows [w_lo, w_hi) need frames
w_lo .. w_hi + 4, i.e. the samples [160 w_lo, 160 (w_hi + 4) + 401) -- a
240-sample + 4-frame overlap with the neighbour's segment, whose duplicated
windows are simply not emitted (each window is classified by exactly one
rank).  The only communication is one gather of the per-window uint8
decisions to rank 0 (RCCL over xGMI when the process group backend is
"nccl"; gloo for the CPU tests).  The reference's only parallelism is the
per-file multiprocessing.Pool of dataset_creator.py:63-65,84.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch
import torch.distributed as dist

FRAME_SIZE = 400
HOP = 160


def shard_range(n_items, rank, world):
    """Contiguous [lo, hi) block of n_items owned by `rank` (sizes differ by <= 1)."""
    base, extra = divmod(n_items, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def n_frames(n_samples, frame_size=FRAME_SIZE, hop=HOP):
    """split_into_frames' count (file_processing.py:99: while len - offset > size)."""
    if n_samples <= frame_size:
        return 0
    return (n_samples - frame_size - 1) // hop + 1


@dataclass(frozen=True)
class ClipShard:
    """Rank `rank`'s part of one clip of n_samples: windows [win_lo, win_hi)
    of the clip's F-5 analyser windows, computed from the samples
    [sample_lo, sample_hi) (a segment whose own framing yields exactly those
    windows: win_hi - win_lo + 5 frames)."""
    rank: int
    world: int
    win_lo: int
    win_hi: int
    sample_lo: int
    sample_hi: int

    @property
    def n_windows(self):
        return self.win_hi - self.win_lo


def split_clip(n_samples, rank, world, frame_size=FRAME_SIZE, hop=HOP):
    """ClipShard of `rank` for a clip of n_samples samples."""
    n_win = max(n_frames(n_samples, frame_size, hop) - 5, 0)
    lo, hi = shard_range(n_win, rank, world)
    if hi <= lo:
        return ClipShard(rank, world, lo, lo, 0, 0)
    # frames lo .. hi + 4 (hi - lo + 5 frames: the last full window is never
    # emitted, file_processing.py:51-70 / sklearn_analyser.py:46-82)
    s_lo = lo * hop
    s_hi = (hi + 4) * hop + frame_size + 1
    return ClipShard(rank, world, lo, hi, s_lo, min(s_hi, n_samples))


def classify_clip_shard(pipe, audio_segment, shard: ClipShard, out=None, stream=None):
    """Labels of this rank's windows from its (already sliced, device) segment."""
    if shard.n_windows == 0:
        return torch.empty((0,), dtype=torch.uint8, device=audio_segment.device)
    if getattr(pipe.cfg, "preemph", None) is not None and shard.sample_lo > 0:
        # the segment's first sample would be pre-emphasised as if it began
        # the clip: apply vad_amd.preemphasis to the whole clip, then shard
        # it with a pipeline whose cfg.preemph is None
        raise ValueError("pre-emphasis must run on the whole clip before sharding")
    lab = pipe.labels(audio_segment, out=out, stream=stream)
    if lab.numel() != shard.n_windows:
        raise ValueError(f"segment of {audio_segment.numel()} samples gives {lab.numel()} windows, "
                         f"shard expects {shard.n_windows}")
    return lab


def _group_dst(dst, group):
    """(group rank of dst, global rank of dst): `dst` is a rank of `group`."""
    if group is None:
        return dst, dst
    return dst, dist.get_global_rank(group, dst)


def gather_labels(labels: torch.Tensor, dst=0, group=None):
    """Gather every rank's 1-D uint8 label tensor to `dst` (a rank of `group`).

    Returns the list of per-rank tensors on `dst` (None elsewhere).  Lengths
    may differ per rank: sizes travel first (a host sync), payloads are
    padded to the max.  Steady-state callers with fixed sizes use
    LabelGather, which allocates once and never syncs the host.
    """
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = labels.device
    n = torch.tensor([labels.numel()], dtype=torch.int64, device=dev)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    sizes = [int(s.item()) for s in sizes]
    m = max(sizes) if sizes else 0
    buf = torch.zeros((max(m, 1),), dtype=torch.uint8, device=dev)
    buf[:labels.numel()].copy_(labels.reshape(-1))
    out = LabelGather(max(m, 1), dev, dst, group)(buf)
    return [o[:s] for o, s in zip(out, sizes)] if rank == dst else None


def any_rank(flag: bool, device=None, group=None) -> bool:
    """True on every rank when `flag` is True on any rank (an all_reduce MAX;
    `device` the backend's: a CUDA device with nccl, the CPU with gloo).  For
    loops whose body holds a collective and whose continuation is decided per
    rank (bench.py's time-based warm-up): agreeing before each trip keeps the
    ranks' collectives matched -- a rank-local decision can leave one rank in
    the loop's collective while another has moved on to the next one."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return bool(flag)
    t = torch.tensor([int(bool(flag))], dtype=torch.int64, device=device or torch.device("cpu"))
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return bool(t.item())


class LabelGather:
    """Gather of a fixed-size uint8 label tensor from every rank to `dst`,
    with the receive buffers allocated once: one collective per call, no
    host synchronisation (the per-step form of bench.py).  With backend
    "nccl" this is RCCL point-to-point (each rank sends its ~1 MB once, to
    dst only, over its own xGMI link).  The collective is chosen once, from
    the backend, identically on every rank: `gather` where the backend
    implements it (nccl, gloo), `all_gather` otherwise -- never a retry after
    a failed collective (ranks would then issue mismatched calls)."""

    GATHER_BACKENDS = ("nccl", "gloo")

    def __init__(self, n, device, dst=0, group=None):
        self.n, self.group = int(n), group
        self.dst, self.global_dst = _group_dst(dst, group)
        self.rank = dist.get_rank(group)  # rank within the group, as dst
        world = dist.get_world_size(group)
        backend = str(dist.get_backend(group)).lower()
        self.use_gather = backend in self.GATHER_BACKENDS
        # gloo collectives take host tensors: device labels are staged through
        # host memory (the CPU tests and the N > 1 rehearsal on one GPU)
        self.via_host = backend == "gloo" and torch.device(device).type == "cuda"
        bdev = "cpu" if self.via_host else device
        self.out = [torch.empty((self.n,), dtype=torch.uint8, device=bdev) for _ in range(world)]

    def __call__(self, labels: torch.Tensor):
        self.start(labels, async_op=False)
        return self.out if self.rank == self.dst else None

    def start(self, labels: torch.Tensor, async_op=True):
        """Issue the gather; with async_op (device buffers, nccl) return its
        work handle at once: the collective runs on the backend's stream after
        the labels are ready, overlapping the caller's next kernels, and
        `handle.wait()` makes the current stream wait for it (no host sync).
        The labels and self.out must not be reused before that wait.  Host-
        staged (gloo) gathers complete before returning (handle None)."""
        if labels.numel() != self.n or labels.dtype != torch.uint8:
            raise ValueError(f"expected {self.n} uint8 labels, got {labels.numel()} {labels.dtype}")
        x = labels.reshape(-1)
        async_op = bool(async_op) and not self.via_host
        if self.via_host:
            x = x.cpu()
        if self.use_gather:
            work = dist.gather(x, self.out if self.rank == self.dst else None, dst=self.global_dst,
                               group=self.group, async_op=async_op)
        else:
            work = dist.all_gather(self.out, x, group=self.group, async_op=async_op)
        return work if async_op else None


def gather_clip_labels(labels: torch.Tensor, shard: ClipShard, dst=0, group=None):
    """Concatenate every rank's window labels of one sharded clip on `dst`
    (the clip's F-5 labels, in order; None elsewhere)."""
    parts = gather_labels(labels, dst, group)
    if parts is None:
        return None
    return torch.cat([p.reshape(-1) for p in parts])


# ----------------------------------------------------------------------------
# The same gather through libvad_amd's C ABI (vad_rccl_*, include/vad_amd.h):
# for hosts without torch.distributed; the unique id travels out of band.
# ----------------------------------------------------------------------------
def rccl_unique_id() -> bytes:
    """ncclGetUniqueId (VAD_RCCL_ID_BYTES bytes) -- on the root rank."""
    import ctypes
    from . import _lib
    buf = ctypes.create_string_buffer(128)
    _lib.check(_lib.lib().vad_rccl_unique_id(buf), "vad_rccl_unique_id")
    return buf.raw


class RcclComm:
    """An RCCL communicator on the current HIP device (vad_rccl_init)."""

    def __init__(self, world, rank, uid: bytes):
        import ctypes
        from . import _lib
        if len(uid) != 128:
            raise ValueError("the RCCL unique id is 128 bytes")
        self.world, self.rank = int(world), int(rank)
        h = ctypes.c_void_p()
        _lib.check(_lib.lib().vad_rccl_init(ctypes.byref(h), self.world, ctypes.create_string_buffer(uid, 128),
                                            self.rank), "vad_rccl_init")
        self._h = h

    def gather_u8(self, send: torch.Tensor, recv: torch.Tensor | None, root=0, stream=None):
        """recv[r * n : (r + 1) * n] = rank r's n uint8 labels, on the root."""
        from . import _lib
        if send.dtype != torch.uint8 or not send.is_cuda or not send.is_contiguous():
            raise TypeError("send must be a contiguous uint8 CUDA tensor")
        if self.rank == root and (recv is None or recv.dtype != torch.uint8
                                  or recv.numel() != self.world * send.numel()):
            raise ValueError("recv must hold world * n uint8 on the root")
        if self.rank == root and (not recv.is_cuda or not recv.is_contiguous() or recv.device != send.device):
            raise TypeError("recv must be a contiguous CUDA tensor on the send tensor's device")
        _lib.check(_lib.lib().vad_rccl_gather_u8(self._h, _lib.ptr(send), _lib.ptr(recv), send.numel(), int(root),
                                                 _lib.stream_ptr(stream)), "vad_rccl_gather_u8")
        return recv

    def close(self):
        from . import _lib
        if getattr(self, "_h", None) is not None and self._h.value:
            _lib.check(_lib.lib().vad_rccl_destroy(self._h), "vad_rccl_destroy")
        self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
