#!/bin/bash
# Counter groups for one kernel under any driver command:
#   bash tools/pmc_kernel.sh OUT KERNEL_REGEX python3 tools/time_apd_pass.py
set -e
OUT=$1; RE=$2; shift 2
mkdir -p $OUT
export TMPDIR=/tmp
for grp in "SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_VMEM_WR TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU" "TA_BUSY_avr TCC_HIT_sum TCC_MISS_sum"; do
  tag=$(echo $grp | cut -d' ' -f1)
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-include-regex "$RE" -d $OUT/v1/$tag -o run --output-format csv -- "$@" > $OUT/$tag.log 2>&1
done
