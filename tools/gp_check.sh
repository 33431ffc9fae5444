#!/bin/bash
# GPU box: APD parity subset, per-kernel A/B (tools/ab_kernels.py) against apde-mvs_amd/lib/ab_head.so, then a
# rocprofv3 kernel-stats pass of the working-tree library:  bash tools/gp_check.sh <outdir> [extra libs...]
OUT=${1:-gpurun_out/gp}; shift
mkdir -p "$OUT"
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q -k "apd or stages or kept or medium or group or f32" --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; [ $rc -le 1 ] || exit $rc
timeout -k 10 400 python3 -u tools/ab_kernels.py apde-mvs_amd/lib/ab_head.so apde-mvs_amd/lib/libapd_hip.so "$@" > "$OUT/k.log" 2>&1 || exit $?
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$OUT/prof" -o run --output-format csv -- python3 "$R/tools/ab_kernels.py" "$R/apde-mvs_amd/lib/libapd_hip.so" > "$R/$OUT/kp.log" 2>&1
