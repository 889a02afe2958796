"""Summarise rocprofv3 counter CSVs: python tools/pmc_sum.py gpurun_out/pmc_<tag> [...]"""
import collections
import csv
import glob
import sys

for d in sys.argv[1:]:
    for f in glob.glob(f"{d}/**/run_counter_collection.csv", recursive=True):
        agg = collections.defaultdict(lambda: collections.defaultdict(list))
        for r in csv.DictReader(open(f)):
            agg[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
        for k, c in agg.items():
            if "vad::" in k:
                print(d.split("/")[-1], k[:60], {n: round(sum(v) / len(v) / 1e6, 2) for n, v in c.items()})
