#!/bin/bash
# Stochastic PC sampling (rocprofv3 beta) of the bench's headline iterations: where the waves of the
# Weak-path kernels stall. Usage (GPU box, repo root): bash tools/pc_sample.sh OUTDIR [interval]
set -e
OUT=$1; IV=${2:-1048576}
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic --pc-sampling-unit cycles \
  --pc-sampling-interval $IV -d "$GRAFT_REPO_ROOT/$OUT/pcs" -o run --output-format csv -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 0 --no-cpu-baseline --end-to-end 0 --c2 0 --rich 0 --sa 0 \
  > "$GRAFT_REPO_ROOT/$OUT/bench.json" 2> "$GRAFT_REPO_ROOT/$OUT/bench.err"
