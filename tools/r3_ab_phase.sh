#!/bin/bash
# GPU: parity subset, C3 A/B against ab_head.so, then the phase profile of the instrumented build.
OUT=${1:-gpurun_out/ab}
mkdir -p "$OUT"
bash tools/r3_ab.sh "$OUT" "${2:-}" || exit $?
APD_LIB=apde-mvs_amd/lib/ab_phase.so timeout -k 10 600 python3 tools/phase_profile.py > "$OUT/phase.txt" 2>&1
cat "$OUT/phase.txt"
