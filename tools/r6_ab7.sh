#!/bin/bash
# Strong sweep at four workgroups per CU (SS_LDS40): GPU parity, then the tree vs SS_LDS40=0 (ab_ss48.so)
# on the texture-rich C3 pass, C2's FIRST_INIT (Strong sweep only) and the smooth C3 headline pass
set -e
O=${1:-gpurun_out/r6ab7}
mkdir -p "$O"
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1
AB_TEXTURE=rich AB_W=6048 AB_H=4032 AB_N=10 AB_FINAL=1 AB_ROUNDS=3 timeout -k 10 400 python3 -u tools/ab_apd.py apde-mvs_amd/lib/ab_ss48.so apde-mvs_amd/lib/libapd_hip.so > "$O/apd_rich.log" 2>&1
AB_FIRST=1 AB_W=3024 AB_H=2016 AB_N=8 AB_ROUNDS=5 timeout -k 10 300 python3 -u tools/ab_apd.py apde-mvs_amd/lib/ab_ss48.so apde-mvs_amd/lib/libapd_hip.so > "$O/c2_first.log" 2>&1
AB_W=6048 AB_H=4032 AB_N=10 AB_FINAL=1 AB_ROUNDS=3 timeout -k 10 400 python3 -u tools/ab_apd.py apde-mvs_amd/lib/ab_ss48.so apde-mvs_amd/lib/libapd_hip.so > "$O/apd.log" 2>&1
echo done
