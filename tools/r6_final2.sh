#!/bin/bash
# Second half of the closing session: rocprofv3 kernel stats of the bench and the PMC summaries.
#   bash tools/r6_final2.sh OUTDIR TAG
set -e
O=${1:-gpurun_out/r6final}
TAG=${2:-r6}
mkdir -p "$O"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
cd /tmp
timeout -k 10 700 rocprofv3 --kernel-trace --stats -d "$R/$O/prof" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu-baseline --c2 0 --rich 0 --sa 0 --steps 6 --warmup 1 > "$R/$O/prof_bench.json" 2> "$R/$O/prof_bench.err"
cd "$R"
bash tools/pmc_round.sh "$O" "$TAG" > "$O/pmc_round.log" 2>&1
echo done > "$O/stage2.ok"
