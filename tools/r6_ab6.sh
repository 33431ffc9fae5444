#!/bin/bash
# texture-rich C3 pass: 6dac4d4 (ab_head.so) vs the tree vs the tree without WV_CUR_MATCH; smooth C3 pass:
# the tree vs RandomInitialization's use_APD instantiation at four waves per SIMD (ab_ri4.so)
set -e
O=${1:-gpurun_out/r6ab6}
mkdir -p "$O"
AB_TEXTURE=rich AB_W=6048 AB_H=4032 AB_N=10 AB_FINAL=1 AB_ROUNDS=3 timeout -k 10 500 python3 -u tools/ab_apd.py apde-mvs_amd/lib/ab_head.so apde-mvs_amd/lib/libapd_hip.so apde-mvs_amd/lib/ab_nomatch.so > "$O/apd_rich.log" 2>&1
AB_W=6048 AB_H=4032 AB_N=10 AB_FINAL=1 AB_ROUNDS=3 timeout -k 10 500 python3 -u tools/ab_apd.py apde-mvs_amd/lib/libapd_hip.so apde-mvs_amd/lib/ab_ri4.so > "$O/apd_ri4.log" 2>&1
echo done
