#!/bin/bash
# A/B against an earlier commit: the library as built from REV's sources (csrc/ + include/, with
# the current build.py flags) under tools/diag/NAME/libballenv.so (git-ignored), e.g.
#   bash tools/build_rev_lib.sh HEAD prev      # then BALLENV_LIB=tools/diag/prev/libballenv.so
set -eu
cd "$(dirname "$0")/.."
rev=$1; name=$2
tmp=$(mktemp -d)
mkdir -p $tmp/gym-ballenv_amd/csrc $tmp/include tools/diag/$name
git archive "$rev" gym-ballenv_amd/csrc include | tar -x -C $tmp
cp gym-ballenv_amd/build.py $tmp/gym-ballenv_amd/build.py
python3 - "$tmp" "$name" <<'PY'
import os, sys
sys.path.insert(0, os.path.join(sys.argv[1], "gym-ballenv_amd"))
import build
build.build_library(force=True, verbose=False, out=os.path.abspath(f"tools/diag/{sys.argv[2]}/libballenv.so"))
PY
rm -rf $tmp
echo "built tools/diag/$name/libballenv.so from $rev"
