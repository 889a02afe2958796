"""Multi-process paths on the GPU box (one MI355X): 2, 3 or 8 ranks sharing
cuda:0 over gloo run the real HIP pipeline on their shard of one clip (the 240-sample
+ 4-frame halo rule) and the gathered labels equal the single-process labels;
a world-size-1 RCCL ("nccl") group runs the label gather bench.py uses.

Ranks are spawned children (fresh interpreters started before they touch the
GPU); RCCL refuses two ranks on one device, so its multi-rank form is left to
the driver's 8-GPU run.
"""
import os
import socket

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

F_CLIP = 200_003


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _clip():
    from oracle import vad_oracle as O
    return O.synth_clip(O.samples_for_frames(F_CLIP), seed=77)


def _pipe():
    from vad_amd.ffn import TOPOLOGY_BL13, FFNClassifier, random_layers
    from vad_amd.pipeline import VadPipeline
    return VadPipeline(FFNClassifier(random_layers(TOPOLOGY_BL13, seed=3)))


def _shard_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist
    from vad_amd.dist import classify_clip_shard, gather_clip_labels, split_clip
    try:
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        clip = _clip()
        sh = split_clip(len(clip), rank, world)
        seg = torch.from_numpy(clip[sh.sample_lo:sh.sample_hi].copy()).cuda()
        pipe = _pipe()
        lab = classify_clip_shard(pipe, seg, sh).cpu()  # gloo gathers host tensors
        full = gather_clip_labels(lab, sh)
        if rank == 0:
            whole = pipe.labels(torch.from_numpy(clip).cuda()).cpu()
            q.put(("ok", int(full.numel()), bool(torch.equal(full, whole)),
                   [(s.win_lo, s.win_hi) for s in (split_clip(len(clip), r, world) for r in range(world))]))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # report instead of hanging the parent
        q.put(("error", repr(e), False, None))
        raise


@pytest.mark.parametrize("world", [2, 3, 8])  # 8: C4's world size, all ranks on cuda:0
def test_clip_shards_on_one_gpu_match_single_process(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_shard_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    status, n, same, ranges = q.get(timeout=150)
    for p in procs:
        p.join(timeout=60)
    assert status == "ok", n
    assert n == F_CLIP - 5 and same, (n, same)
    assert ranges[0][0] == 0 and ranges[-1][1] == F_CLIP - 5
    assert all(a[1] == b[0] for a, b in zip(ranges, ranges[1:]))
    assert all(p.exitcode == 0 for p in procs)


def _rccl_worker(port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1")
    import torch
    import torch.distributed as dist
    from vad_amd.dist import LabelGather, gather_labels
    try:
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        dist.init_process_group("nccl", device_id=dev)
        assert dist.get_backend() == "nccl"
        g = torch.Generator(device="cuda").manual_seed(5)
        lab = torch.randint(0, 3, (1_000_000,), dtype=torch.uint8, device=dev, generator=g)
        lg = LabelGather(lab.numel(), dev)
        got = lg(lab)
        torch.cuda.synchronize()
        ok1 = lg.use_gather and len(got) == 1 and bool(torch.equal(got[0], lab))
        var = gather_labels(lab[:12345])
        ok2 = len(var) == 1 and bool(torch.equal(var[0], lab[:12345]))
        # bench.py's overlapped form: two buffers, the gather of one running
        # on RCCL's stream while the next labels are written to the other
        from vad_amd.pipeline import VadPipeline
        from vad_amd.ffn import FFNClassifier, TOPOLOGY_BL13, random_layers
        pipe = VadPipeline(FFNClassifier(random_layers(TOPOLOGY_BL13, seed=2)))
        audio = torch.randn(160 * 20_000 + 241, generator=g, device=dev) * 3000
        n = pipe.n_frames(audio.numel()) - 5
        bufs = [torch.empty(n, dtype=torch.uint8, device=dev) for _ in range(2)]
        gs = [LabelGather(n, dev) for _ in range(2)]
        pend = [None, None]
        ref = pipe.labels(audio).clone()
        for step in range(6):
            i = step % 2
            if pend[i] is not None:
                pend[i].wait()
            pipe.labels(audio, out=bufs[i])
            pend[i] = gs[i].start(bufs[i], async_op=True)
        for w in pend:
            w.wait()
        torch.cuda.synchronize()
        ok2 = ok2 and all(bool(torch.equal(gg.out[0], ref)) for gg in gs)
        dist.destroy_process_group()
        q.put(("ok", ok1, ok2))
    except Exception as e:
        q.put(("error", repr(e), False))
        raise


def test_rccl_world1_label_gather():
    """RCCL (torch "nccl" backend on ROCm) group of one: LabelGather picks
    gather from the backend and returns the rank's 1M labels unchanged."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_worker, args=(_free_port(), q))
    p.start()
    status, ok1, ok2 = q.get(timeout=150)
    p.join(timeout=60)
    assert status == "ok", ok1
    assert ok1 and ok2
    assert p.exitcode == 0


def _capi_worker(q):
    import torch
    from vad_amd.dist import RcclComm, rccl_unique_id
    try:
        torch.cuda.set_device(0)
        comm = RcclComm(1, 0, rccl_unique_id())
        g = torch.Generator(device="cuda").manual_seed(6)
        lab = torch.randint(0, 2, (1_000_000,), dtype=torch.uint8, device="cuda", generator=g)
        recv = torch.empty_like(lab)
        comm.gather_u8(lab, recv)
        torch.cuda.synchronize()
        ok = bool(torch.equal(recv, lab))
        comm.close()
        q.put(("ok", ok))
    except Exception as e:
        q.put(("error", repr(e)))
        raise


def test_capi_rccl_world1_gather():
    """vad_rccl_unique_id / _init / _gather_u8 / _destroy (the C-ABI form of
    the label gather, RCCL resolved at run time) on a group of one."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_capi_worker, args=(q,))
    p.start()
    status, ok = q.get(timeout=150)
    p.join(timeout=60)
    assert status == "ok" and ok is True, ok
    assert p.exitcode == 0


def test_bench_gpus_launches_ranks():
    """`bench.py --gpus 2` with no launcher starts the two rank processes
    itself (torch.distributed.run on 127.0.0.1): rank 0 prints one JSON line
    with n_gpus 2 and the gather object (gloo: both ranks share the one GPU
    of the test box)."""
    import json
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--backend", "gloo",
                        "--frames", "20000", "--steps", "2", "--warmup", "1", "--no-cpu", "--no-secondary",
                        "--min-warmup-s", "0.05"],
                       capture_output=True, text=True, timeout=240, env=env, cwd=REPO)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["parallelism"] == "clip-shard x2"
    assert out["gather"]["label_bytes_per_rank"] == 20000 - 5 and out["gather"]["backend"] == "gloo"
    assert out["value"] > 0
