"""No kernel of the library depends on what an earlier kernel left in LDS.

LDS is not cleared between launches: a kernel that reads a word it did not
write first sees whatever the previous kernel on that CU left there.  The
fused clip kernel did (its first tile's halo rows, found by the fuzz tests:
tests/test_gpu_fused.py::test_fused_independent_of_stale_lds).  Here every
compute entry is run once on clean inputs and again right after a test-only
kernel (tests/c_host/lds_poison.hip) filled every CU's 160 KB of LDS with a
hostile value (+-1e30, past f16 and any feature range; NaN); the outputs
must be bit-identical: MFCC (compiled 26 / 40-filter banks, runtime tables,
int16 PCM, another FFT length), spectra, window features, the FFN window
kernel (split-f16 topologies, 3 classes, exact f32, with logits), the fused
kernel, the decision tree, the streaming hop kernel (one hop and blocks of
8) and the three-kernel step, and SimpleAnalyser features.
"""
import ctypes
import os

import numpy as np
import pytest

from oracle import vad_oracle as O

pytestmark = pytest.mark.gpu

POISON = (1e30, -1e30, float("nan"))


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    return torch


@pytest.fixture(scope="module")
def poison(torch_cuda):
    torch = torch_cuda
    so = os.path.join(os.path.dirname(os.path.abspath(__file__)), "c_host", "liblds_poison.so")
    if not os.path.exists(so):
        pytest.fail("tests/c_host/liblds_poison.so missing: run __graft_entry__.build()")
    helper = ctypes.CDLL(so)
    helper.lds_poison.argtypes = [ctypes.c_float, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    sink = torch.zeros(1, device="cuda")
    n_cu = torch.cuda.get_device_properties(0).multi_processor_count

    def fill(v):
        st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        assert helper.lds_poison(v, ctypes.c_void_p(sink.data_ptr()), 4 * n_cu, st) == 0

    yield fill
    torch.cuda.synchronize()
    v = sink.item()
    assert v == 0.0  # every poison launch read back its own LDS stores


def bits(t):
    """A comparable copy of a result (a tensor, numpy array, or tuple of them):
    bit patterns, so NaN outputs compare equal to themselves."""
    import torch
    if isinstance(t, (tuple, list)):
        return [bits(x) for x in t]
    if isinstance(t, np.ndarray):
        t = torch.from_numpy(np.ascontiguousarray(t))
    t = t.detach().contiguous().cpu()
    if t.dtype in (torch.float32, torch.int32):
        return t.view(torch.int32).clone()
    if t.dtype in (torch.float64, torch.int64):
        return t.view(torch.int64).clone()
    return t.clone()


def same(a, b):
    import torch
    if isinstance(a, list):
        return all(same(x, y) for x, y in zip(a, b))
    return torch.equal(a, b)


def check(fill, name, fn):
    want = bits(fn())
    for v in POISON:
        fill(v)
        assert same(bits(fn()), want), (name, v)


def test_clip_kernels_ignore_stale_lds(torch_cuda, poison):
    torch = torch_cuda
    from vad_amd import _lib
    from vad_amd.ffn import TOPOLOGY_BL13, TOPOLOGY_REF39, FFNClassifier, random_layers
    from vad_amd.pipeline import VadPipeline
    from vad_amd.plan import MfccPlan, window_features, window_logits
    clip = O.synth_clip(O.samples_for_frames(5000), seed=31)
    clip[160 * 2000:160 * 2100] = 0.0  # digital silence: NaN features, flagged windows
    a = torch.from_numpy(clip).cuda()
    a16 = a.to(torch.int16)
    for nf in (26, 40):
        plan = MfccPlan(O.get_mel_filterbanks(300, 8000, 512, nf, 16000))
        check(poison, f"mfcc{nf}", lambda: plan.clip_mfcc(a))
        check(poison, f"mfcc{nf} int16", lambda: plan.clip_mfcc(a16))
        plan.set_variant(0)
        check(poison, f"mfcc{nf} runtime tables", lambda: plan.clip_mfcc(a))
    p1024 = MfccPlan(O.get_mel_filterbanks(300, 8000, 1024, 26, 16000), 13, 1024)
    check(poison, "mfcc fft 1024", lambda: p1024.clip_mfcc(a[:160 * 300]))
    frames = a[:400 * 64].reshape(64, 400)
    plan26 = MfccPlan(O.get_mel_filterbanks(300, 8000, 512, 26, 16000))
    check(poison, "spec", lambda: plan26.spec(frames))
    m = plan26.clip_mfcc(a)
    for mode in (_lib.FEAT_ANALYSER, _lib.FEAT_OFFLINE):
        check(poison, f"features {mode}", lambda: window_features(m, mode))
    for topo in (TOPOLOGY_BL13, TOPOLOGY_REF39, (13, 64, 64, 3)):
        for arith in ("split", "f32"):
            clf = FFNClassifier(random_layers(topo, seed=3), **({"arith": "f32"} if arith == "f32" else {}))
            check(poison, f"ffn {topo} {arith}", lambda: clf.plan.window_labels(m))
            check(poison, f"ffn logits {topo} {arith}", lambda: window_logits(clf.plan, m))
        for mode in ("analyser", "offline"):
            pipe = VadPipeline(FFNClassifier(random_layers(topo, seed=3)), mode=mode)
            check(poison, f"two-kernel {topo} {mode}", lambda: pipe.labels(a))
            check(poison, f"fused {topo} {mode}", lambda: pipe.labels(a, fused=True))


def test_tree_and_simple_ignore_stale_lds(torch_cuda, golden, poison):
    torch = torch_cuda
    from sklearn.tree import DecisionTreeClassifier
    from vad_amd.plan import MfccPlan
    from vad_amd.simple_analyser import SimpleAnalyser
    from vad_amd.tree import TreeClassifier
    gt = golden("tree")
    clf = DecisionTreeClassifier(max_depth=25, min_samples_leaf=5, random_state=0).fit(
        np.nan_to_num(gt["x_test"]), gt["y_test"])
    tree = TreeClassifier.from_sklearn(clf)
    clip = O.synth_clip(O.samples_for_frames(3000), seed=32)
    a = torch.from_numpy(clip).cuda()
    m = MfccPlan(O.get_mel_filterbanks(300, 8000, 512, 26, 16000)).clip_mfcc(a)
    check(poison, "tree windows", lambda: tree.window_labels(m))
    x = torch.from_numpy(np.nan_to_num(gt["x_test"]).astype(np.float32)).cuda()
    check(poison, "tree rows", lambda: tree.predict_device(x))
    sa = SimpleAnalyser(16000, 400, 5)
    fr = clip[:400 * 200].reshape(200, 400)
    check(poison, "simple features", lambda: sa.frame_features(fr))


@pytest.mark.parametrize("kernel,K", [("hop", 1), ("hop", 8), ("three", 1)])
def test_stream_kernels_ignore_stale_lds(torch_cuda, golden, poison, kernel, K):
    """T hops through a clean batch and through one whose every launch is
    preceded by a poison launch: identical labels and state."""
    torch = torch_cuda
    from vad_amd.ffn import FFNClassifier
    from vad_amd.stream import StreamBatch
    w = golden("ffn")
    clf = FFNClassifier([(w[f"ref39_W{i}"], w[f"ref39_b{i}"]) for i in range(4)])
    S, T = 300, 16
    clips = np.stack([O.synth_clip(160 * (T - 1) + 401, seed=900 + s) for s in range(S)])
    carry = torch.from_numpy(np.ascontiguousarray(clips[:, :240])).cuda()
    hops = torch.from_numpy(np.ascontiguousarray(
        np.stack([clips[:, 240 + 160 * t: 400 + 160 * t] for t in range(T)]))).cuda()
    outs = []
    for v in (None,) + POISON:
        sb = StreamBatch(S, clf, kernel=kernel, hops_per_step=K)
        sb.prime(carry)
        labs = []
        for t in range(0, T, K):
            if v is not None:
                poison(v)
            labs.append((sb.step(hops[t]) if K == 1 else sb.step_block(hops[t:t + K])).clone())
        outs.append(bits([torch.stack(labs), sb.frames, sb.ring, sb.count]))
    for o in outs[1:]:
        assert same(o, outs[0])
