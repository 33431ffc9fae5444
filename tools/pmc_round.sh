#!/bin/bash
# PMC summaries of the C3 headline's kernels at the current tree (GPU box, repo root):
#   bash tools/pmc_round.sh OUTDIR TAG
# tools/pmc_c3.sh's counter passes (end to end included, so the prepare-phase and DepthToWeak kernels
# run too), then one tools/pmc_json.py summary per kernel, OUTDIR/TAG_pmc_<kernel>_c3.json, each
# carrying the kernel sources' hash recorded at collection time (bench.py reports traffic only from a
# summary whose hash matches the tree it runs from).
set -e
OUT=${1:-gpurun_out/pmc_round}
TAG=${2:-r6}
RE="k_sweep_weak_vm|k_weak_cand_g|k_weak_cand_comb|k_gp_cost|k_gp_dedup|k_gp_count_loc|k_gen_anchors|k_depth_to_weak_vm|k_sweep_strong_vm|k_random_init_vm"
bash tools/pmc_c3.sh "$OUT/pmc" "$RE" --end-to-end 1 > "$OUT/pmc.log" 2>&1
for k in k_sweep_weak_vm k_weak_cand_g k_weak_cand_comb k_gp_cost k_gp_dedup_q k_gp_count_loc k_gen_anchors_fit "k_gen_anchors<" k_depth_to_weak_vm k_sweep_strong_vm "k_random_init_vm<true, true"; do
  name=$(echo "$k" | tr -d '<, ' | sed 's/truetrue/_apd/')
  python3 tools/pmc_json.py "$OUT/pmc" "$OUT/${TAG}_pmc_${name}_c3.json" --kernel "$k" --width 6048 --height 4032 --n-src 10 \
    --source "rocprofv3 --pmc, one pass per counter group (tools/pmc_c3.sh via tools/pmc_round.sh), bench.py --steps 3 --warmup 0 --end-to-end 1 at C3" > /dev/null
done
echo done
