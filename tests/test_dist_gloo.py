"""world_size-2 gloo test of the clip-sharding gather (CPU; the GPU run uses
RCCL through the same code with backend "nccl")."""
import os
import socket

import numpy as np
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
    # the asynchronous form bench.py overlaps with the next step (two
    # buffers, each reused after its handle's wait)
    gs = [LabelGather(4, torch.device("cpu")) for _ in range(2)]
    bufs = [torch.empty(4, dtype=torch.uint8) for _ in range(2)]
    pend = [None, None]
    for step in range(4):
        i = step % 2
        if pend[i] is not None:
            pend[i].wait()
            if rank == 0:
                q.put([t.tolist() for t in gs[i].out])
        bufs[i].fill_(rank * 10 + step)
        pend[i] = gs[i].start(bufs[i], async_op=True)
        assert pend[i] is not None
    for i in range(2):
        pend[i].wait()
        if rank == 0:
            q.put([t.tolist() for t in gs[i].out])
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 8])  # 8: the driver's C4 world size, rehearsed on gloo
def test_gather_labels_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    fixed = [q.get(timeout=120) for _ in range(2)]
    overlapped = [q.get(timeout=120) for _ in range(4)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert got == [(i * 3) % 7 for i in range(11)]
    for step, f in enumerate(fixed):
        assert f == [[r * 10 + step] * 4 for r in range(world)]
    for step, f in enumerate(overlapped):
        assert f == [[r * 10 + step] * 4 for r in range(world)]


def test_split_clip_covers_every_window_once():
    from oracle import vad_oracle as O
    from vad_amd.dist import split_clip
    for F in (6, 7, 100, 1001, 1_000_000):
        L = O.samples_for_frames(F)
        for world in (1, 2, 3, 8):
            shards = [split_clip(L, r, world) for r in range(world)]
            assert shards[0].win_lo == 0 and shards[-1].win_hi == F - 5
            for a, b in zip(shards, shards[1:]):
                assert a.win_hi == b.win_lo
            for s in shards:
                if s.n_windows:
                    # the segment's own framing yields exactly its windows + 5 frames
                    assert O.n_frames(s.sample_hi - s.sample_lo) == s.n_windows + 5
                    assert s.sample_lo == 160 * s.win_lo and s.sample_hi <= L


def _oracle_shard_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import vad_oracle as O
    from vad_amd.dist import gather_clip_labels, split_clip
    from vad_amd.ffn import TOPOLOGY_BL13, random_layers
    layers = random_layers(TOPOLOGY_BL13, seed=3)
    fb = O.get_mel_filterbanks(300, 8000, 512, 26, 16000)
    clip = O.synth_clip(O.samples_for_frames(3001), seed=12)
    sh = split_clip(len(clip), rank, world)

    def labels(x):
        return O.ffn_labels(O.analyser_features_fast(O.mfcc_batch(x, fb))[:, :13], layers)
    lab = torch.from_numpy(labels(clip[sh.sample_lo:sh.sample_hi]).astype(np.uint8))
    full = gather_clip_labels(lab, sh)
    if rank == 0:
        q.put(bool(np.array_equal(full.numpy(), labels(clip).astype(np.uint8))))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 8])
def test_sharded_clip_labels_equal_whole_clip(world):
    """The halo rule on the CPU oracle: every rank classifies its segment,
    the gathered labels are the whole clip's (windows at every cut included)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_oracle_shard_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    same = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert same


def _warmup_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from vad_amd.dist import LabelGather, any_rank
    g = LabelGather(4, torch.device("cpu"))
    # bench.py's warm-up shape: every trip holds a collective (the step's
    # gather) and the continuation is rank-local (here: rank r wants 2 + 2r
    # trips); any_rank makes every rank run the longest rank's trips
    trips = 0
    while any_rank(trips < 2 + 2 * rank):
        g(torch.full((4,), rank, dtype=torch.uint8))
        trips += 1
    q.put((rank, trips))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 8])
def test_warmup_continuation_agreed_across_ranks(world):
    """Regression (the 2-rank bench rehearsal hung when the ranks' time-based
    warm-up ran different numbers of gathering steps): with any_rank every
    rank runs the same number of trips, so the collectives stay matched."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_warmup_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert got == {r: 2 + 2 * (world - 1) for r in range(world)}
