"""A/B of the wave-private MFCC prototype (tools/micro/wp_proto.hip) against
the shipped mfcc_kernel, on one box, in one process:

    python tools/wp_ab.py [variant[:wg_per_cu] ...]   (default "-:3": tools/bin/libwp_proto.so, 3 per CU)

Checks the prototype's MFCC rows against the shipped kernel's (bit for bit
expected: same FFT code, same per-filter chains, same MFMA DCT) on C3 (1M
frames) and C2 (100k), then times both, interleaved, as the median of 9
batches of 20 launches after a 0.5 s warm-up.  Prints one JSON line."""
import ctypes
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import synth_audio  # noqa: E402
from vad_amd import _lib  # noqa: E402
from vad_amd.pipeline import VadPipeline  # noqa: E402

# variants: "name[:wg_per_cu]" -> tools/bin/libwp_proto[_name].so ("-" = the default build)
protos = {}
for spec in sys.argv[1:] or ["-:3"]:
    name, _, w = spec.partition(":")
    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "bin", "libwp_proto.so" if name == "-" else f"libwp_proto_{name}.so"))
    lib.wp_mfcc.restype = ctypes.c_int
    lib.wp_mfcc.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_longlong, ctypes.c_void_p, ctypes.c_int,
                            ctypes.c_void_p]
    protos[f"{name}w{w or 3}"] = (lib, int(w or 3))

dev = torch.device("cuda", 0)
pipe = VadPipeline()


def wp(a, out, key):
    lib, wgpc = protos[key]
    rc = lib.wp_mfcc(pipe.plan.handle, a.data_ptr(), out.shape[0], out.data_ptr(), wgpc, _lib.stream_ptr())
    assert rc == 0, rc


def median_us(fn, batches=9, reps=20):
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.5:
        fn()
    torch.cuda.synchronize()
    out = []
    for _ in range(batches):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            fn()
        e.record()
        torch.cuda.synchronize()
        out.append(s.elapsed_time(e) / reps * 1e3)
    out.sort()
    return out[len(out) // 2], out


res = {}
for name, F in (("c3", 1_000_000), ("c2", 100_000)):
    a = synth_audio(160 * (F - 1) + 401, 1, dev)
    ref = torch.empty((F, 13), device=dev)
    pipe.mfcc(a, out=ref)
    for key in protos:
        got = torch.full((F, 13), float("nan"), device=dev)
        wp(a, got, key)
        torch.cuda.synchronize()
        same = (got == ref) | (torch.isnan(got) & torch.isnan(ref))
        d = (got - ref).abs().max(dim=1).values / ref.abs().max(dim=1).values
        res[f"{name}_{key}_check"] = {"bit_equal_frac": same.float().mean().item(),
                                        "rows_differing": int((~same.all(dim=1)).sum().item()),
                                        "max_rel_row_diff": float(torch.nan_to_num(d, nan=0.0).max().item()),
                                        "nan_rows": int(torch.isnan(got).any(dim=1).sum().item())}
    for rnd in range(2):  # interleaved: shipped, prototype(s), shipped, ...
        res.setdefault(f"{name}_shipped_us", []).append(median_us(lambda: pipe.mfcc(a, out=ref))[0])
        for key in protos:
            res.setdefault(f"{name}_{key}_us", []).append(median_us(lambda: wp(a, got, key))[0])
    del a, ref, got
    torch.cuda.empty_cache()
print(json.dumps(res))
