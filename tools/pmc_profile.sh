#!/bin/bash
# PMC passes on the Strong sweep kernel (run on the GPU box from the repo root):
#   bash tools/pmc_profile.sh <outdir> [kernel-regex]
# One rocprofv3 process per counter group (counters only, no sys/runtime tracing), each bounded by
# its own timeout; stops at the first failure. Summarise with tools/pmc_summarize.py <outdir>.
set -e
OUT=${1:-gpurun_out/pmc}
RE=${2:-k_sweep_strong}
mkdir -p "$OUT"
export TMPDIR=/tmp
CMD="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --end-to-end 0"
i=0
for grp in \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU" \
  "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM" \
  "TA_BUSY_avr TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum" \
  "FETCH_SIZE" \
  "WRITE_SIZE" ; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-include-regex "$RE" -d "$OUT/p$i" -o run --output-format csv -- $CMD > "$OUT/p$i.log" 2>&1
done
echo done
