#!/bin/bash
# The whole C3-shaped scan at C3's N = 10 (GPU box, repo root): 26 views at 6048x4032, pair.txt capped at
# 10 sources per view, no SA masks, main.cpp's full schedule through the `apd` binary; per-pass loop-body
# rates from the library's phase timing (APD_PHASE_TIMING). Usage: bash tools/scan_c3_n10.sh OUTDIR [prof]
# With `prof` the scene is written first and rocprofv3 runs the apd binary itself (no launcher hop).
set -e
OUT=$1
mkdir -p "$OUT"
export TMPDIR=/tmp TIME_SCAN_SA=0 TIME_SCAN_NSRC=10
if [ "$2" = prof ]; then
  F=/tmp/apd_scan_c3_n10
  TIME_SCAN_FOLDER=$F TIME_SCAN_RUN=0 timeout -k 10 600 python3 -u tools/time_scan.py 6048 4032 26 > "$OUT/scene.txt" 2>&1
  APD="$GRAFT_REPO_ROOT/apde-mvs_amd/host/build/apd"
  cd /tmp
  APD_PHASE_TIMING=1 timeout -k 10 1000 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run --output-format csv -- "$APD" -d $F --dataset ETH3D --no_fuse true > "$GRAFT_REPO_ROOT/$OUT/apd_stdout.log" 2>&1
  cd "$GRAFT_REPO_ROOT"
  python3 tools/time_scan.py --parse "$OUT/apd_stdout.log" 6048 4032 26 > "$OUT/scan.txt" 2>&1
else
  TIME_SCAN_LOG="$GRAFT_REPO_ROOT/$OUT/apd_stdout.log" timeout -k 10 1100 python3 -u tools/time_scan.py 6048 4032 26 > "$OUT/scan.txt" 2>&1
fi
