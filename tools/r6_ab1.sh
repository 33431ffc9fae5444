#!/bin/bash
# Round-6 A/B session (GPU box, repo root): parity tests of the working tree, then the headline APD pass
# at C3 for HEAD (ab_head.so), the working tree and variants, and the instrumented phase profile.
set -e
O=${1:-gpurun_out/r6ab1}
mkdir -p "$O"
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1
AB_W=6048 AB_H=4032 AB_N=10 AB_FINAL=1 AB_ROUNDS=3 timeout -k 10 500 python3 -u tools/ab_apd.py apde-mvs_amd/lib/ab_head.so apde-mvs_amd/lib/libapd_hip.so ${AB_EXTRA} > "$O/apd.log" 2>&1
APD_LIB=apde-mvs_amd/lib/ab_phase.so timeout -k 10 300 python3 -u tools/phase_profile.py > "$O/phase.log" 2>&1
echo done
