#!/bin/bash
# PMC passes on the C3 headline's Weak-path kernels (run on the GPU box from the repo root):
#   bash tools/pmc_c3.sh <outdir> [kernel-regex] [bench args...]
# One rocprofv3 process per counter group (counters only, no sys/runtime tracing), each bounded by
# its own timeout; stops at the first failure. Summarise with tools/pmc_json.py.
set -e
OUT=${1:-gpurun_out/pmc_c3}
RE=${2:-"k_sweep_weak_vm|k_weak_cand_g|k_gp_cost"}
EXTRA="${*:3}"
mkdir -p "$OUT"
# the kernel sources' hash at collection time (bench.py source_hash): tools/pmc_json.py stores it in the
# summary, and bench.py reports the summary's traffic only while the tree still has these sources
python3 -c "import bench; print(bench.source_hash())" > "$OUT/source_hash"
export TMPDIR=/tmp
CMD="python3 bench.py --steps 3 --warmup 0 --no-cpu-baseline --end-to-end 0 --c2 0 --rich 0 --sa 0 $EXTRA"
i=0
for grp in \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU" \
  "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM" \
  "TA_BUSY_avr TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum" \
  "FETCH_SIZE" \
  "WRITE_SIZE" ; do
  i=$((i+1))
  echo "[$(date +%T)] pass $i: $grp"
  timeout -k 10 400 rocprofv3 --pmc $grp --kernel-include-regex "$RE" -d "$OUT/p$i" -o run --output-format csv -- $CMD > "$OUT/p$i.log" 2>&1
done
echo done
