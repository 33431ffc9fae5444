#!/bin/bash
# Device-resident state of the apd binary (GPU box, repo root): CLI parity tests, then the same
# synthetic scan with APD_DEVICE_STATE=1 (default) and =0 (host uploads), host breakdowns side by side.
#   bash tools/r3_devstate.sh <outdir> [W H VIEWS]
OUT=${1:-gpurun_out/devstate}
W=${2:-3024}; H=${3:-2016}; V=${4:-11}
mkdir -p "$OUT"
export TMPDIR=/tmp APD_HOST_TIMING=1
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_cli.py -v --timeout 300 --timeout-method thread > "$OUT/pytest_cli.log" 2>&1
rc=$?; echo "pytest rc=$rc" >> "$OUT/steps.log"
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
for ds in 1 0; do
  APD_DEVICE_STATE=$ds TIME_SCAN_LOG="$OUT/apd_ds$ds.log" timeout -k 10 900 python3 -u tools/time_scan.py $W $H $V > "$OUT/scan_ds$ds.txt" 2>&1 || exit $?
  echo "scan ds=$ds done" >> "$OUT/steps.log"
done
echo ok
