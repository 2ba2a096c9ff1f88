#!/bin/bash
# Round 5, third A/B session: step2_kernel with 16 envs per wave (2 waves per SIMD at 32 768 envs;
# lanes 32..63 shadow 0..31) against 32 (in-tree), at 32 768 and 65 536 envs.  Timing only: the
# 16-env build's stats slots race (two waves per 32-env slot).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
B="epw16" REPS=3 bash tools/legs_ab.sh || exit 1
echo done
