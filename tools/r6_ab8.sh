#!/bin/bash
# k_gp_count_loc with per-workgroup aggregation (GP_LOC_BLOCK): GPU parity, then the bench's headline line
# (pairs_ms_per_pass, prepare timings) for the tree and for GP_LOC_BLOCK=0 (ab_loc0.so), twice each
set -e
O=${1:-gpurun_out/r6ab8}
mkdir -p "$O"
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1
B="python3 -u bench.py --steps 6 --warmup 1 --no-cpu-baseline --c2 0 --rich 0 --sa 0 --end-to-end 0"
APD_LIB=apde-mvs_amd/lib/ab_loc0.so timeout -k 10 300 $B > "$O/loc0_a.json" 2> "$O/loc0_a.err"
timeout -k 10 300 $B > "$O/loc1_a.json" 2> "$O/loc1_a.err"
APD_LIB=apde-mvs_amd/lib/ab_loc0.so timeout -k 10 300 $B > "$O/loc0_b.json" 2> "$O/loc0_b.err"
timeout -k 10 300 $B > "$O/loc1_b.json" 2> "$O/loc1_b.err"
echo done
