#!/bin/bash
# Round-6 A/B session 2 (GPU box, repo root): DepthToWeak's inner-band statistics, the whole GPU suite,
# then the C3 headline pass for HEAD (ab_head.so), the working tree and the tree without the early decision.
set -e
O=${1:-gpurun_out/r6ab2}
mkdir -p "$O"
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
timeout -k 10 600 python3 -u tools/dtw_early_stats.py > "$O/dtw_early.log" 2>&1
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > "$O/pytest.log" 2>&1
AB_W=6048 AB_H=4032 AB_N=10 AB_FINAL=1 AB_ROUNDS=3 timeout -k 10 500 python3 -u tools/ab_apd.py apde-mvs_amd/lib/ab_head.so apde-mvs_amd/lib/libapd_hip.so apde-mvs_amd/lib/ab_noearly.so > "$O/apd.log" 2>&1
echo done
