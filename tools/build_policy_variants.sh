#!/bin/bash
# Diagnostics builds of libballenv.so with other policy tile counts (BE_POL_TILES) -> tools/diag/
set -e
cd "$(dirname "$0")/.."
mkdir -p tools/diag
# each argument: NAME:FLAGS, e.g. T2:-DBE_POL_TILES=2  T2u:"-DBE_POL_TILES=2 -DBE_POL_UNROLL=13"
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -shared -ffp-contract=off -fno-fast-math --offload-arch=gfx950 \
      $flags -I include gym-ballenv_amd/csrc/ballenv.hip -o tools/diag/libballenv_$name.so &
done
wait
