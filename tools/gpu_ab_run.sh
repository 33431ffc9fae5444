#!/bin/bash
# GPU A/B step (run on the box from the repo root): parity tests, then the working-tree library
# against apde-mvs_amd/lib/ab_head.so (tools/build_head.sh) on the Strong sweep, a FIRST_INIT
# RunPatchMatch and an APD pass. Each step has its own time limit; stops at the first failure.
set -e
OUT=${1:-gpurun_out/ab}
mkdir -p "$OUT"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
AB_ROUNDS=5 timeout -k 10 300 python3 -u tools/ab_sweep.py apde-mvs_amd/lib/ab_head.so apde-mvs_amd/lib/libapd_hip.so > "$OUT/sweep.log" 2>&1
AB_ROUNDS=5 timeout -k 10 300 python3 -u tools/ab_e2e.py apde-mvs_amd/lib/ab_head.so apde-mvs_amd/lib/libapd_hip.so > "$OUT/e2e.log" 2>&1
AB_ROUNDS=3 timeout -k 10 400 python3 -u tools/ab_apd.py apde-mvs_amd/lib/ab_head.so apde-mvs_amd/lib/libapd_hip.so > "$OUT/apd.log" 2>&1
echo done
