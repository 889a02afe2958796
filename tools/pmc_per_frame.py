"""Per-launch and per-frame PMC values of the bench's kernels from a
tools/profile.sh run: python tools/pmc_per_frame.py gpurun_out/prof_<tag> > profiles/<tag>_pmc.txt
(first 3 launches of each kernel skipped as warm-up; 1M frames / windows per launch)."""
import collections
import csv
import glob
import sys

d = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{d}/**/run_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for label, key in (("mfcc_kernel (fp32, 26 mel, paired frames), per 1M-frame launch",
                    "mfcc_kernel<float, 0, 13, true, 400, 1, 5, false>"),
                   ("mfcc_kernel (int16 PCM), per 1M-frame launch", "mfcc_kernel<short, 0, 13, true, 400, 1, 5, false>"),
                   ("ffn_wave_kernel (13-64-64-2 split-f16), per 1M-window launch", "ffn_wave_kernel<4, 4, 4, 1, 0, 2, 0, false>"),
                   ("ffn_wave_group_kernel (13-64-64-2 tile pairs), per 1M-window launch", "ffn_wave_group_kernel<0, 2>"),
                   ("mfcc_ffn_kernel (fused, 13-64-64-2), per 1M-frame launch", "mfcc_ffn_kernel<float")):
    ks = [k for k in agg if key in k]
    if not ks:
        continue
    print(f"== {label}")
    for n in sorted(agg[ks[0]]):
        v = agg[ks[0]][n]
        v = v[3:] if len(v) > 6 else v
        m = sum(v) / len(v)
        print(f"{n:28s} {m:14.6g}   per frame {m / 1e6:10.4g}")
