#!/bin/bash
# The C3 N=10 scan twice on one box: the default LDS Weak sweep, then APD_WEAK_REC=1 (anchor records,
# four workgroups per CU). Usage: bash tools/scan_rec_vs_lds.sh OUTDIR
set -e
OUT=$1
mkdir -p "$OUT"
export TMPDIR=/tmp TIME_SCAN_SA=0 TIME_SCAN_NSRC=10
F=/tmp/apd_scan_c3_n10
TIME_SCAN_FOLDER=$F TIME_SCAN_RUN=0 timeout -k 10 600 python3 -u tools/time_scan.py 6048 4032 26 > "$OUT/scene.txt" 2>&1
APD=apde-mvs_amd/host/build/apd
for v in lds rec; do
  if [ $v = rec ]; then export APD_WEAK_REC=1; fi
  APD_PHASE_TIMING=1 timeout -k 10 500 $APD -d $F --dataset ETH3D --no_fuse true > "$OUT/apd_$v.log" 2>&1
  python3 tools/time_scan.py --parse "$OUT/apd_$v.log" 6048 4032 26 > "$OUT/scan_$v.txt" 2>&1
done
