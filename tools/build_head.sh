#!/bin/bash
# Build libapd_hip.so from a git revision (default HEAD) into OUT, for A/B against the working tree:
#   bash tools/build_head.sh OUT.so [REV] [extra hipcc flags...]
set -e
OUT=$1; REV=${2:-HEAD}; shift 2 || shift $#
D=$(mktemp -d)
mkdir -p $D/apde-mvs_amd/csrc $D/include
for f in apd_kernels.hip apd_fusion.hip apd_device.h; do git show $REV:apde-mvs_amd/csrc/$f > $D/apde-mvs_amd/csrc/$f; done
for f in apd_hip.h apd_fusion.h; do git show $REV:include/$f > $D/include/$f; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -w -shared "$@" \
  -o "$OUT" $D/apde-mvs_amd/csrc/apd_kernels.hip $D/apde-mvs_amd/csrc/apd_fusion.hip
rm -rf $D
