#!/bin/bash
# A/B library builds (git-ignored) under tools/diag/<name>/libballenv.so: each arg "name:-DFLAG=v -DFLAG2=v"
set -eu
cd "$(dirname "$0")/.."
F="-O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math --offload-arch=gfx950 -mllvm -amdgpu-mfma-vgpr-form -I include"
for spec in "$@"; do
  n=${spec%%:*}; d=${spec#*:}
  mkdir -p tools/diag/$n
  /opt/rocm/bin/hipcc $F -shared $d gym-ballenv_amd/csrc/ballenv.hip gym-ballenv_amd/csrc/policy.hip \
      gym-ballenv_amd/csrc/features.hip gym-ballenv_amd/csrc/board.hip -o tools/diag/$n/libballenv.so 2>&1 | grep -E "error" &
done
wait
echo built
