set -e
OUT=gpurun_out/r3_ab2; mkdir -p $OUT
AB_W=6048 AB_H=4032 AB_N=10 AB_FINAL=1 AB_ROUNDS=2 timeout -k 10 500 python3 -u tools/ab_apd.py apde-mvs_amd/lib/libapd_hip.so apde-mvs_amd/lib/ab_randlocal.so > $OUT/apd_c3.log 2>&1
AB_W=6048 AB_H=4032 AB_N=10 AB_FIRST=1 AB_ROUNDS=2 timeout -k 10 500 python3 -u tools/ab_apd.py apde-mvs_amd/lib/libapd_hip.so apde-mvs_amd/lib/ab_randlocal.so > $OUT/first_c3.log 2>&1
AB_W=3024 AB_H=2016 AB_N=8 AB_FIRST=1 AB_ROUNDS=3 timeout -k 10 300 python3 -u tools/ab_apd.py apde-mvs_amd/lib/libapd_hip.so apde-mvs_amd/lib/ab_randlocal.so > $OUT/first_c2.log 2>&1
cat $OUT/*.log
