#!/bin/bash
# A/B on the GPU box (repo root): the working-tree library against apde-mvs_amd/lib/ab_head.so
# (tools/build_head.sh) on the APD parity cases and the C3 headline pass (tools/ab_apd.py).
#   bash tools/r3_ab.sh <outdir> [pytest -k expression]
OUT=${1:-gpurun_out/ab}
K=${2:-}
mkdir -p "$OUT"
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q ${K:+-k "$K"} --timeout 400 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { echo "pytest failed: $?"; tail -30 "$OUT/pytest.log"; exit 1; }
AB_W=6048 AB_H=4032 AB_N=10 AB_FINAL=1 AB_ROUNDS=3 timeout -k 10 500 python3 -u tools/ab_apd.py apde-mvs_amd/lib/ab_head.so apde-mvs_amd/lib/libapd_hip.so > "$OUT/apd_c3.log" 2>&1
AB_W=6048 AB_H=4032 AB_N=10 AB_FIRST=1 AB_ROUNDS=2 timeout -k 10 500 python3 -u tools/ab_apd.py apde-mvs_amd/lib/ab_head.so apde-mvs_amd/lib/libapd_hip.so > "$OUT/first_c3.log" 2>&1
AB_W=3024 AB_H=2016 AB_N=8 AB_FIRST=1 AB_ROUNDS=3 timeout -k 10 300 python3 -u tools/ab_apd.py apde-mvs_amd/lib/ab_head.so apde-mvs_amd/lib/libapd_hip.so > "$OUT/first_c2.log" 2>&1
cat "$OUT"/*_c*.log
