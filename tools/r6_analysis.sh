set -e
mkdir -p gpurun_out/r6s7
APD_LIB=apde-mvs_amd/lib/ab_phase.so timeout -k 10 300 python3 -u tools/phase_profile.py > gpurun_out/r6s7/phase.txt 2>&1
bash tools/pmc_c3.sh gpurun_out/r6s7/pmc "k_sweep_weak_vm|k_gp_dedup|k_gen_anchors|k_depth_to_weak_vm|k_sweep_strong_vm|k_gp_count_loc|k_weak_cand_g|k_weak_cand_comb|k_gp_cost" --end-to-end 1 > gpurun_out/r6s7/pmc.log 2>&1
echo ok
