"""Per-window PMC of the 13-64-64-2 FFN kernels from tools/pmc_ffn_ab.sh:
python tools/pmc_ffn_report.py gpurun_out/<tag> NAME...  (medians over launches
after the first three; SQ counters summed over the device, per 1M-window launch,
divided by the launch's windows)."""
import collections
import csv
import glob
import json
import statistics
import sys

out = {}
d = sys.argv[1]
for v in sys.argv[2:]:
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"{d}/{v}/**/run_counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0]
            if "ffn_wave" not in k:
                continue
            agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    res = {}
    for k, ctr in agg.items():
        res[k] = {c: round(statistics.median(vals[3:] or vals) / 999_995, 3) for c, vals in ctr.items()}
    out[v] = res
print(json.dumps(out, indent=1))
