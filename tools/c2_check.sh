#!/bin/bash
# Default bench (with the secondary configs) twice; prints the C2 lines.
set -u
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/c2
mkdir -p $OUT
cd $R
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --no-cpu > $OUT/bench_$r.json 2> $OUT/bench_$r.err || { tail -20 $OUT/bench_$r.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_$r.json'));s=d['secondary_configs'];print({k:(round(v.get('avg_launch_us',v.get('us_per_batch',0)),2),round(v['frac_hbm'],3)) for k,v in s.items() if k.startswith('c2')}, d['ms_per_step'])"
done
