#!/bin/bash
# Round-6 analysis session (GPU box, repo root): parity first, then the Weak sweep's phase profile
# (instrumented build apde-mvs_amd/lib/ab_phase.so, -DAPD_PHASE_STAMPS) and PMC passes over the
# prepare-phase and loop-body kernels at C3 (tools/pmc_c3.sh, end to end included).
set -e
O=${1:-gpurun_out/r6s7}
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/parity.log 2>&1
APD_LIB=apde-mvs_amd/lib/ab_phase.so timeout -k 10 300 python3 -u tools/phase_profile.py > $O/phase.txt 2>&1
bash tools/pmc_c3.sh $O/pmc "k_sweep_weak_vm|k_gp_dedup|k_gen_anchors|k_depth_to_weak_vm|k_sweep_strong_vm|k_gp_count_loc|k_weak_cand_g|k_weak_cand_comb|k_gp_cost" --end-to-end 1 > $O/pmc.log 2>&1
echo ok
