"""Mean per-launch counter values of the MFCC kernel from tools/pmc_passes.sh output:
python tools/pmc_report.py <tag> [kernel-substring]"""
import collections
import csv
import glob
import sys

tag = sys.argv[1]
kname = sys.argv[2] if len(sys.argv) > 2 else "mfcc_kernel"
res = {}
for f in sorted(glob.glob(f"gpurun_out/pmc_{tag}_*/**/run_counter_collection.csv", recursive=True)):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if kname in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in agg.items():
        v = v[3:] if len(v) > 6 else v  # skip warm-up launches
        res[k] = sum(v) / len(v)
for k in sorted(res):
    print(f"{k:32s} {res[k]:.4g}")
