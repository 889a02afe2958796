"""Per-frame PMC values per kernel from tools/pmc_ab.sh output:
python tools/pmc_summary.py gpurun_out/pmcab_<tag> [frames_per_launch]"""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1]
frames = float(sys.argv[2]) if len(sys.argv) > 2 else 1e6
for lib in sorted(os.listdir(root)):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"{root}/{lib}/**/run_counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            agg[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, ctr in agg.items():
        if "mfcc" not in k:
            continue
        print(f"== {lib}: {k}")
        for n in sorted(ctr):
            v = ctr[n][20:] if len(ctr[n]) > 40 else ctr[n]
            m = sum(v) / len(v)
            print(f"  {n:28s} {m:14.6g}   per frame {m / frames:10.4g}")
