set -e
mkdir -p gpurun_out/ab2
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ab2/pytest.log 2>&1
AB_ROUNDS=5 timeout -k 10 300 python3 -u tools/ab_e2e.py apde-mvs_amd/lib/ab_head.so apde-mvs_amd/lib/libapd_hip.so > gpurun_out/ab2/e2e.log 2>&1
AB_ROUNDS=3 timeout -k 10 400 python3 -u tools/ab_apd.py apde-mvs_amd/lib/ab_head.so apde-mvs_amd/lib/libapd_hip.so > gpurun_out/ab2/apd.log 2>&1
echo done
