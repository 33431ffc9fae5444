#!/bin/bash
# Counter comparison of the Strong sweep under two environments: bash tools/pmc_ab.sh OUT "ENV_A" "ENV_B"
set -e
OUT=$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for envs in "$@"; do
  i=$((i+1))
  for grp in "SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_VMEM_WR TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU" "TA_BUSY_avr TA_TA_BUSY_sum TD_BUSY_sum" ; do
    tag=$(echo $grp | cut -d' ' -f1)
    env $envs timeout -k 10 200 rocprofv3 --pmc $grp --kernel-include-regex k_sweep_strong -d $OUT/v$i/$tag -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --end-to-end 0 > $OUT/v$i.$tag.log 2>&1
  done
done
