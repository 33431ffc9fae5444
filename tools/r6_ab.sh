#!/bin/bash
# Round-6 A/B session (GPU box, repo root): the GPU parity tests of the working tree, then the C3
# headline pass for HEAD (ab_head.so), the working tree and the variants given as arguments.
#   bash tools/r6_ab.sh OUTDIR [variant.so ...]
set -e
O=${1:-gpurun_out/r6ab}
shift || true
mkdir -p "$O"
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1
AB_W=6048 AB_H=4032 AB_N=10 AB_FINAL=1 AB_ROUNDS=3 timeout -k 10 600 python3 -u tools/ab_apd.py apde-mvs_amd/lib/ab_head.so apde-mvs_amd/lib/libapd_hip.so "$@" > "$O/apd.log" 2>&1
echo done
