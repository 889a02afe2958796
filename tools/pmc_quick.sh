#!/bin/bash
# One PMC pass over the bench: tools/pmc_quick.sh <tag> "<counters>" [env...]
set -u
TAG=$1; CTRS=$2
cd /tmp && export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_$TAG
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --pmc $CTRS -d $OUT -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu > $OUT/log 2>&1
