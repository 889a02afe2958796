#!/bin/bash
# Kernel trace + PMC passes of the bench on the GPU box.
#   tools/profile.sh <tag> [bench args...]
# Writes gpurun_out/prof_<tag>/{trace,pmc1..4}/ ; each pass runs under its own timeout.
set -u
TAG=$1; shift
ARGS=${@:---steps 5 --warmup 2 --no-cpu}
cd /tmp && export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py $ARGS > $OUT/trace.log 2>&1 || exit 1
# the same on one stream: no dispatch waits for CUs held by the other
# stream's kernels, so the stats' per-kernel averages are kernel durations
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace1 -o run --output-format csv -- python3 bench.py $ARGS --streams 1 > $OUT/trace1.log 2>&1 || exit 6
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE -d $OUT/pmc1 -o run --output-format csv -- python3 bench.py $ARGS > $OUT/pmc1.log 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS -d $OUT/pmc2 -o run --output-format csv -- python3 bench.py $ARGS > $OUT/pmc2.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc3 -o run --output-format csv -- python3 bench.py $ARGS > $OUT/pmc3.log 2>&1 || exit 4
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc4 -o run --output-format csv -- python3 bench.py $ARGS > $OUT/pmc4.log 2>&1 || exit 5
echo profile done
