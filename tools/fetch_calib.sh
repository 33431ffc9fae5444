#!/bin/bash
# FETCH_SIZE calibration on the GPU box (repo root): bash tools/fetch_calib.sh OUTDIR
# Pass 0: timings; pass 1: FETCH_SIZE; pass 2: the raw L2->fabric read requests (64 B and 32 B).
set -e
OUT=$1
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 120 ./tools/fetch_calib > "$OUT/timing.jsonl" 2> "$OUT/timing.err"
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$GRAFT_REPO_ROOT/$OUT/p1" -o run --output-format csv -- "$GRAFT_REPO_ROOT/tools/fetch_calib" > "$GRAFT_REPO_ROOT/$OUT/p1.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum -d "$GRAFT_REPO_ROOT/$OUT/p2" -o run --output-format csv -- "$GRAFT_REPO_ROOT/tools/fetch_calib" > "$GRAFT_REPO_ROOT/$OUT/p2.log" 2>&1
cd "$GRAFT_REPO_ROOT"
python3 tools/fetch_calib_summary.py "$OUT" > "$OUT/summary.json"
