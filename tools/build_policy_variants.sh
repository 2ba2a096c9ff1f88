#!/bin/bash
# Diagnostics builds of libballenv.so with extra compile flags -> tools/diag/libballenv_<NAME>.so
# each argument: NAME:FLAGS, e.g. nofma:-DSOME_DIAG_FLAG=1
set -e
cd "$(dirname "$0")/.."
mkdir -p tools/diag
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  python3 -c "import sys; sys.path.insert(0, '.'); from gym_ballenv_amd.build import build_library; \
build_library(verbose=False, extra_flags='$flags'.split(), out='tools/diag/libballenv_$name.so')" &
done
wait
