#!/bin/bash
# UTCL1 (address translation) and TCP counters of the Strong sweep at C2 and C3 sizes
set -e
OUT=${1:-gpurun_out/tcp_sizes}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 --list-avail > $OUT/avail.txt 2>&1 || true
for cfg in "3024 2016 8" "6048 4032 8"; do
  set -- $cfg
  timeout -k 10 300 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum --kernel-include-regex k_sweep_strong -d $OUT/p_$1 -o run --output-format csv -- python3 bench.py --width $1 --height $2 --n-src $3 --steps 2 --warmup 1 --no-cpu-baseline --end-to-end 0 --apd-pass 0 > $OUT/p_$1.log 2>&1
done
echo done
