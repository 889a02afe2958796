"""world_size-2 gloo test of the clip-sharding gather (CPU; the GPU run uses
RCCL through the same code with backend "nccl")."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from vad_amd.dist import gather_labels, shard_range
    n_items = 11
    lo, hi = shard_range(n_items, rank, world)
    labels = torch.arange(lo, hi, dtype=torch.uint8) * 3 % 7
    out = gather_labels(labels)
    if rank == 0:
        q.put(torch.cat(out).tolist())
    # fixed-size, preallocated form (bench.py's per-step gather), twice
    from vad_amd.dist import LabelGather
    g = LabelGather(4, torch.device("cpu"))
    for step in range(2):
        got = g(torch.full((4,), rank * 10 + step, dtype=torch.uint8))
        if rank == 0:
            q.put([t.tolist() for t in got])
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gather_labels_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    fixed = [q.get(timeout=120) for _ in range(2)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert got == [(i * 3) % 7 for i in range(11)]
    for step, f in enumerate(fixed):
        assert f == [[r * 10 + step] * 4 for r in range(world)]
