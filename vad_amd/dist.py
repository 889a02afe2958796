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
    may differ per rank: sizes travel first, payloads are padded to the max.
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
    if dist.get_backend(group) == "nccl":
        # RCCL gather = all_gather into rank-ordered slots (payload ~1 MB/rank)
        out = [torch.empty_like(buf) for _ in range(world)]
        dist.all_gather(out, buf, group=group)
        return [o[:s] for o, s in zip(out, sizes)] if rank == dst else None
    out = [torch.empty_like(buf) for _ in range(world)] if rank == dst else None
    dist.gather(buf, out, dst=dst, group=group)
    return [o[:s] for o, s in zip(out, sizes)] if rank == dst else None
