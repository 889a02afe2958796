"""[Historical: the diagnostic hooks this needs were removed from the shipped kernels in round 4;
build it from a tree at or before commit 4f8ce33.]  Per-workgroup start/end stamps of mfcc_kernel (a -DVAD_DIAG_BUILD=9 library): shader clock,
workgroup durations vs kernel wall time, dispatch skew."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
# the stamps come from a diagnostic library build (the shipped one has none):
#   python -m vad_amd.build --variant diag9 -DVAD_DIAG_BUILD=9
os.environ.setdefault("VAD_AMD_LIB", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                  "vad_amd", "lib", "libvad_amd_diag9.so"))
os.environ.setdefault("VAD_DIAG", "9")  # read by this script only
from bench import synth_audio  # noqa: E402
from vad_amd.pipeline import VadPipeline  # noqa: E402

pipe = VadPipeline()
F = int(os.environ.get("VAD_FRAMES", "1000000"))
audio = synth_audio(160 * (F - 1) + 401, 1, torch.device("cuda"))
buf = torch.zeros(F * 13 + 1024 * 8, dtype=torch.float32, device="cuda")
out = buf[: F * 13].view(F, 13)
for _ in range(150):
    pipe.mfcc(audio, out=out)
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
pipe.mfcc(audio, out=out)
e.record()
torch.cuda.synchronize()
wall_us = s.elapsed_time(e) * 1e3
st = buf[F * 13:].view(torch.int64).cpu().numpy().reshape(1024, 4).astype(np.float64)
blk = np.nonzero(st[:, 1] > 0)[0]
st = st[st[:, 1] > 0]  # launched workgroups
t0, r0, t1, r1 = st[:, 0], st[:, 1], st[:, 2], st[:, 3]
clk = (t1 - t0) / ((r1 - r0) / 100e6) / 1e9  # s_memrealtime: 100 MHz
dur_us = (r1 - r0) / 100.0
start_us = (r0 - r0.min()) / 100.0
end_us = (r1 - r0.min()) / 100.0
print(f"wall {wall_us:.1f} us; shader clock median {np.median(clk):.3f} GHz (min {clk.min():.3f} max {clk.max():.3f})")
print(f"workgroup duration us: min {dur_us.min():.1f} median {np.median(dur_us):.1f} max {dur_us.max():.1f}")
print(f"start skew us: max {start_us.max():.1f}; end spread: first {end_us.min():.1f} last {end_us.max():.1f}")
print("workgroups", len(st), "cycles per workgroup: median", np.median(t1 - t0))
cyc = t1 - t0
print(f"cycles per workgroup: min {cyc.min():.0f} max {cyc.max():.0f}")
for x in range(8):  # workgroups are dealt to the 8 XCDs round-robin (block b -> XCD b mod 8)
    m = blk % 8 == x
    print(f"XCD {x}: clock {np.median(clk[m]):.3f} GHz, duration median {np.median(dur_us[m]):.1f} "
          f"max {dur_us[m].max():.1f} us, cycles median {np.median(cyc[m]):.0f}")
