"""Per-phase kernel durations from a rocprofv3 --kernel-trace of bench.py
(tools/profile.sh output):  python tools/trace_phase_stats.py gpurun_out/prof_<tag> [last_n]

bench.py alternates consecutive steps over two HIP streams, so in the warm-up
and timed steps one step's MFCC kernel overlaps the previous step's MFCC tail
and FFN: those dispatches' start-to-end durations include time shared with
the other stream, and rocprof's overall average (run_kernel_stats.csv) mixes
them in.  The bench's per-kernel `kernels_ms` (and roofline.avg_launch_ms)
come from events around back-to-back launches on ONE stream after the timed
region: the last `last_n` dispatches of each kernel (10 = one event batch in
tools/profile.sh's --steps 5 run).  This prints, per kernel, the average of
those last dispatches, their launch-to-launch period (what the events see,
dispatch gaps included), and the average over the earlier, overlapped ones."""
import collections
import csv
import json
import re
import sys

d = sys.argv[1]
last_n = int(sys.argv[2]) if len(sys.argv) > 2 else 10
rows = collections.defaultdict(list)
for r in csv.DictReader(open(f"{d}/trace/run_kernel_trace.csv")):
    rows[r["Kernel_Name"]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Stream_Id"])))
bench = {}
try:
    m = re.search(r"^\{.*\}$", open(f"{d}/trace.log").read(), re.M)
    bench = json.loads(m.group(0)).get("kernels_ms", {}) if m else {}
except (OSError, ValueError):
    pass
out = {"last_n": last_n, "bench_kernels_ms": bench, "kernels": {}}
for name, v in sorted(rows.items(), key=lambda kv: -sum(e - s for s, e, _ in kv[1])):
    if len(v) < last_n + 1 or not ("mfcc_kernel" in name or "ffn_wave_kernel" in name or "ffn_wave_group_kernel" in name or "mfcc_ffn_kernel" in name):
        continue
    v.sort()
    tail, head = v[-last_n:], v[:-last_n]
    dur = lambda xs: sum(e - s for s, e, _ in xs) / len(xs) / 1e3
    period = (tail[-1][1] - tail[0][0]) / len(tail) / 1e3
    out["kernels"][name] = {"dispatches": len(v), "last_n_avg_us": dur(tail), "last_n_period_us": period,
                            "last_n_streams": sorted({s for _, _, s in tail}),
                            "earlier_avg_us": dur(head), "earlier_streams": sorted({s for _, _, s in head})}
print(json.dumps(out, indent=1))
