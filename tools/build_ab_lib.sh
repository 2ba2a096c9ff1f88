#!/bin/bash
# A/B library builds (git-ignored, under tools/diag/<name>/libballenv.so): the whole library from the
# current sources with extra defines, e.g.  bash tools/build_ab_lib.sh boardold -DBE_BOARD_NO_FAST_RESET
#                                           bash tools/build_ab_lib.sh st -DBE_DIAG_STAMPS
set -eu
cd "$(dirname "$0")/.."
name=$1; shift
mkdir -p tools/diag/$name
F="-O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math --offload-arch=gfx950 -I include -I gym-ballenv_amd/csrc"
/opt/rocm/bin/hipcc $F "$@" -shared gym-ballenv_amd/csrc/ballenv.hip gym-ballenv_amd/csrc/policy.hip \
    gym-ballenv_amd/csrc/features.hip gym-ballenv_amd/csrc/board.hip -o tools/diag/$name/libballenv.so 2>/dev/null
echo "built tools/diag/$name/libballenv.so"
