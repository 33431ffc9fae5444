#!/bin/bash
# The whole C3-shaped scan at C3's N = 10 (GPU box, repo root): 26 views at 6048x4032, pair.txt capped at
# 10 sources per view, no SA masks, main.cpp's full schedule through the `apd` binary; per-pass loop-body
# rates from the library's phase timing. Usage: bash tools/scan_c3_n10.sh OUTDIR [prof]
set -e
OUT=$1
mkdir -p "$OUT"
export TMPDIR=/tmp TIME_SCAN_SA=0 TIME_SCAN_NSRC=10 TIME_SCAN_LOG="$GRAFT_REPO_ROOT/$OUT/apd_stdout.log"
if [ "$2" = prof ]; then
  cd /tmp
  timeout -k 10 1100 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/time_scan.py" 6048 4032 26 > "$GRAFT_REPO_ROOT/$OUT/scan.txt" 2>&1
else
  timeout -k 10 1100 python3 -u tools/time_scan.py 6048 4032 26 > "$OUT/scan.txt" 2>&1
fi
