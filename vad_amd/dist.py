"""Multi-GPU clip sharding (BASELINE config 4).

Independent clips shard across ranks with no data-path collective: rank r
classifies its own clips on its own GPU.  The only communication is one
gather of the per-window uint8 decisions to rank 0 (RCCL over xGMI when the
process group backend is "nccl"; gloo for the CPU tests).
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def shard_range(n_items, rank, world):
    """Contiguous [lo, hi) block of n_items owned by `rank` (sizes differ by <= 1)."""
    base, extra = divmod(n_items, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def gather_labels(labels: torch.Tensor, dst=0, group=None):
    """Gather every rank's 1-D uint8 label tensor to `dst`.

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
    buf = torch.zeros((m,), dtype=torch.uint8, device=dev)
    buf[:labels.numel()].copy_(labels.reshape(-1))
    out = LabelGather(m, dev, dst, group)(buf)
    return [o[:s] for o, s in zip(out, sizes)] if rank == dst else None


class LabelGather:
    """Gather of a fixed-size uint8 label tensor from every rank to `dst`,
    with the receive buffers allocated once: one collective per call, no
    host synchronisation (the per-step form of bench.py).  With backend
    "nccl" this is RCCL point-to-point (each rank sends its ~1 MB once, to
    dst only, over its own xGMI link); should the backend refuse gather the
    call falls back to all_gather into the same slots."""

    def __init__(self, n, device, dst=0, group=None):
        self.n, self.dst, self.group = int(n), dst, group
        self.rank = dist.get_rank(group)
        world = dist.get_world_size(group)
        self.out = [torch.empty((self.n,), dtype=torch.uint8, device=device) for _ in range(world)]
        self._use_gather = True

    def __call__(self, labels: torch.Tensor):
        if labels.numel() != self.n or labels.dtype != torch.uint8:
            raise ValueError(f"expected {self.n} uint8 labels, got {labels.numel()} {labels.dtype}")
        x = labels.reshape(-1)
        if self._use_gather:
            try:
                dist.gather(x, self.out if self.rank == self.dst else None, dst=self.dst,
                            group=self.group)
                return self.out if self.rank == self.dst else None
            except (RuntimeError, NotImplementedError):
                self._use_gather = False
        dist.all_gather(self.out, x, group=self.group)
        return self.out if self.rank == self.dst else None
