#!/bin/bash
# L1/L2/TA counters of the Strong sweep for several library builds:
#   bash tools/pmc_libs.sh OUT lib1.so lib2.so ...   (summarise with tools/pmc_ab_sum.py-style reads)
set -e
OUT=$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for lib in "$@"; do
  i=$((i+1))
  for grp in "SQ_INSTS_VMEM_RD TCP_TCC_READ_REQ_sum TA_BUSY_avr TCC_HIT_sum TCC_MISS_sum" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_BUSY_CU_CYCLES SQ_WAVES"; do
    tag=$(echo $grp | cut -d' ' -f1)
    APD_LIB=$lib timeout -k 10 200 rocprofv3 --pmc $grp --kernel-include-regex k_sweep_strong -d $OUT/v$i/$tag -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --end-to-end 0 > $OUT/v$i.$tag.log 2>&1
  done
done
echo done
