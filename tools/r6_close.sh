#!/bin/bash
# Round-6 closing session in one call (GPU box, repo root): the PMC summaries at the tree's kernel-source
# hash, the default bench line, a rocprofv3 kernel-stats run of the bench, smoke() and the whole GPU suite.
# Every step has its own time limit; the script stops at the first failure.
#   bash tools/r6_close.sh OUTDIR TAG
set -e
O=${1:-gpurun_out/r6close}
TAG=${2:-r6}
mkdir -p "$O"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
bash tools/pmc_round.sh "$O" "$TAG" > "$O/pmc_round.log" 2>&1
timeout -k 10 400 python3 -u bench.py > "$O/bench.json" 2> "$O/bench.err"
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/$O/prof" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu-baseline --c2 0 --rich 0 --sa 0 --steps 6 --warmup 1 > "$R/$O/prof_bench.json" 2> "$R/$O/prof_bench.err"
cd "$R"
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
timeout -k 10 420 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1
echo done > "$O/close.ok"
