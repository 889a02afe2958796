#!/bin/bash
# Matrix-core MFCC kernel: GPU test suite (all tests, failures listed), then a short bench.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04b
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" $O/tests.log | tail -30
case $rc in 0|1) ;; *) echo "pytest rc $rc"; exit 10;; esac
timeout -k 10 300 python3 bench.py --no-cpu --no-secondary --steps 50 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 11; }
python3 -c "
import json; d=json.load(open('$O/bench.json'))
print('value', d['value'], 'ms', d['ms_per_step'], d.get('ms_per_step_serial'))
print('kernels', d['kernels_ms'])
print('roofline', d['roofline'])"
timeout -k 10 400 python3 tools/ab_mfcc.py vad_amd/lib/libvad_amd.so vad_amd/lib/libvad_amd_nopar.so vad_amd/lib/libvad_amd_noperm.so vad_amd/lib/libvad_amd_valu.so 2 > $O/ab.json 2>&1 || { tail -5 $O/ab.json; exit 12; }
cat $O/ab.json
