"""Co-residency probe (tools/micro/coresident.hip): the MFCC kernel (1M frames)
alone, an FFN-shaped filler (32 MFMA + 256 VALU per tile, 60 VGPRs, no LDS,
1024 waves = 4 per CU) alone, and the two launched together on two streams
(MFCC first).  Prints per-iteration microseconds of each arm."""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.getcwd())
from bench import synth_audio  # noqa: E402
from vad_amd.pipeline import VadPipeline  # noqa: E402

dev = torch.device("cuda", 0)
pipe = VadPipeline()
F = 1_000_000
a = synth_audio(160 * (F - 1) + 401, 1, dev)
m = torch.empty((F, 13), device=dev)
fl = ctypes.CDLL(os.path.join(os.getcwd(), "bin_tmp", "libcoresident.so"))
fl.filler_launch.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
blocks = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
tiles = int(sys.argv[2]) if len(sys.argv) > 2 else 61
fout = torch.empty(blocks * 64, device=dev)
sa = torch.cuda.current_stream()
sb = torch.cuda.Stream(device=dev)


def mfcc():
    pipe.mfcc(a, out=m)


def filler(stream):
    fl.filler_launch(fout.data_ptr(), blocks, tiles, ctypes.c_void_p(stream.cuda_stream))


def timed(fn, reps=50, warm=100):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record(sa)
    for _ in range(reps):
        fn()
    sa.wait_stream(sb)  # the end event covers the second stream's work too
    e.record(sa)
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def both():
    # independent work: the filler on the second stream is not ordered after
    # the MFCC launch, so the two may share the CUs
    mfcc()
    filler(sb)


def serial():
    mfcc()
    filler(sa)


sb.wait_stream(sa)
res = {"blocks": blocks, "tiles": tiles}
for r in range(3):
    res.setdefault("mfcc_alone", []).append(timed(mfcc))
    res.setdefault("filler_alone", []).append(timed(lambda: filler(sa)))
    res.setdefault("serial_same_stream", []).append(timed(serial))
    res.setdefault("concurrent_two_streams", []).append(timed(both))
print(json.dumps(res))
