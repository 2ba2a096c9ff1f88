#!/bin/bash
# A/B library builds (git-ignored, under tools/diag/<name>/libballenv.so): the whole library from the
# current sources through build.py (its per-unit flags included) with extra defines, e.g.
#   bash tools/build_ab_lib.sh ct128 -DBE_S2_CT=128
#   bash tools/build_ab_lib.sh st -DBE_DIAG_STAMPS
set -eu
cd "$(dirname "$0")/.."
name=$1; shift
mkdir -p tools/diag/$name
python3 - "$name" "$@" <<'PY'
import os, sys
sys.path.insert(0, "gym-ballenv_amd")
import build
build.build_library(force=True, verbose=False, extra_flags=tuple(sys.argv[2:]),
                    out=os.path.abspath(f"tools/diag/{sys.argv[1]}/libballenv.so"))
PY
echo "built tools/diag/$name/libballenv.so"
