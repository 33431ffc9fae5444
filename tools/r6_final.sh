#!/bin/bash
# A round's closing GPU session (GPU box, repo root): the whole -m gpu suite, smoke(), the default bench
# line, a rocprofv3 kernel-stats run of the bench, and the PMC summaries of the C3 kernels
# (tools/pmc_round.sh). Every step has its own time limit; the script stops at the first failure.
#   bash tools/r6_final.sh OUTDIR TAG
set -e
O=${1:-gpurun_out/r6final}
TAG=${2:-r6}
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 1500 python3 -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > "$O/pytest_gpu.log" 2>&1
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
timeout -k 10 900 python3 -u bench.py > "$O/bench.json" 2> "$O/bench.err"
echo done > "$O/stage1.ok"
