#!/bin/bash
# One GPU-box pass (run from the repo root): gpu parity tests, smoke, bench, rocprofv3 kernel stats.
#   bash tools/gpu_check.sh <outdir> [tests|bench|all]
# Each GPU step has its own time limit; the script stops at the first failure.
set -e
OUT=${1:-gpurun_out/check}
WHAT=${2:-all}
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ "$WHAT" = tests ] || [ "$WHAT" = all ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
  timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
fi
if [ "$WHAT" = bench ] || [ "$WHAT" = all ]; then
  timeout -k 10 600 python3 -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
  cd /tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline --end-to-end 0 --c2 0 --rich 0 --steps 6 --warmup 1 > "$GRAFT_REPO_ROOT/$OUT/prof_bench.json" 2> "$GRAFT_REPO_ROOT/$OUT/prof_bench.err"
fi
echo ok
