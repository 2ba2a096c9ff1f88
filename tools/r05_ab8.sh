#!/bin/bash
# Round-5 A/B of a step2 variant library (V, under tools/diag/V): its step2 parity tests through
# BALLENV_LIB, then the headline / config-2 / config-4 shard legs interleaved with the in-tree build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
V=${V:?variant}; O=gpurun_out/r05_ab8_$V; mkdir -p $O
BALLENV_LIB=tools/diag/$V/libballenv.so timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_gpu_episode.py} -k "${K:-step2 or default_episode}" -m gpu -x -q -p no:cacheprovider --timeout 150 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
B="$V" REPS=${REPS:-3} bash tools/legs_ab.sh
