#!/bin/bash
# Load-path PMC passes over the MFCC kernel, fp32 vs int16 input:
#   tools/pmc_load.sh   (writes gpurun_out/pmcl_<dtype>_<pass>/)
set -u
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
PASSES=(
  "GRBM_GUI_ACTIVE TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum"
  "TA_DATA_STALLED_BY_TC_CYCLES_sum TA_ADDR_STALLED_BY_TD_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum"
  "TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum"
  "TCP_TCC_READ_REQ_LATENCY_sum TCP_TOTAL_CACHE_ACCESSES_sum"
  "TCP_UTCL1_TRANSLATION_MISS_sum TCP_TCR_TCP_STALL_CYCLES_sum"
  "TCP_READ_TAGCONFLICT_STALL_CYCLES_sum SQ_WAIT_INST_ANY SQ_BUSY_CYCLES"
)
for dt in f32 i16; do
  i=0
  for P in "${PASSES[@]}"; do
    OUT=$R/gpurun_out/pmcl_${dt}_$i
    mkdir -p $OUT
    if [ $dt = i16 ]; then export VAD_DIAG_INT16=1; else unset VAD_DIAG_INT16; fi
    timeout -k 10 100 rocprofv3 --pmc $P -d $OUT -o run --output-format csv -- python3 $R/tools/diag_time.py > $OUT/log 2>&1 || exit $?
    i=$((i+1))
  done
done
