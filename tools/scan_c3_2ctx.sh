#!/bin/bash
# The C3-shaped N = 10 scan (26 views at 6048x4032, no SA, main.cpp's full schedule, Jacobi passes) through
# the `apd` binary with one context (--gpus 0) and with two contexts on the same GPU (--gpus 0,0: two
# problems in flight, each context with its own device store, the pass's maps exchanged at the commit),
# the reference's --work_num in one process (run.py:16, 82). GPU box, repo root:
#   bash tools/scan_c3_2ctx.sh OUTDIR
set -e
OUT=$1
mkdir -p "$OUT"
export TMPDIR=/tmp TIME_SCAN_SA=0 TIME_SCAN_NSRC=10
F=/tmp/apd_scan_c3_n10
TIME_SCAN_FOLDER=$F TIME_SCAN_RUN=0 timeout -k 10 600 python3 -u tools/time_scan.py 6048 4032 26 > "$OUT/scene.txt" 2>&1
APD="$GRAFT_REPO_ROOT/apde-mvs_amd/host/build/apd"
for cfg in "0" "0,0"; do
  tag=gpus_${cfg/,/_}
  echo "[$(date +%T)] --gpus $cfg --ordering jacobi"
  rm -rf "$F/APD"
  s=$(date +%s%N)
  APD_PHASE_TIMING=1 timeout -k 10 900 "$APD" -d $F --dataset ETH3D --no_fuse true --gpus $cfg --ordering jacobi > "$OUT/$tag.log" 2>&1
  e=$(date +%s%N)
  echo "wall_s $(( (e - s) / 1000000 ))e-3" > "$OUT/$tag.wall"
  python3 tools/time_scan.py --parse "$OUT/$tag.log" 6048 4032 26 > "$OUT/$tag.txt" 2>&1
  for v in 00000000 00000013 00000025; do md5sum $F/APD/$v/depths.bin $F/APD/$v/normals.bin $F/APD/$v/weak.bin >> "$OUT/$tag.md5"; done
done
# Jacobi outputs do not depend on the number of contexts: the two runs' files must be identical
cmp <(cut -d' ' -f1 "$OUT/gpus_0.md5") <(cut -d' ' -f1 "$OUT/gpus_0_0.md5") && echo "outputs identical" >> "$OUT/gpus_0_0.wall"
echo done
