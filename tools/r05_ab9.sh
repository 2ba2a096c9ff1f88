#!/bin/bash
# Round-5 whole-library change: the full GPU suite, then 3x interleaved A/Bs of the step-API legs
# (legs_ab.sh: headline / config 2 / config-4 shard) and the one-lane legs (big_ab.sh) against tools/diag/$B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05_m}; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 150 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
B="${B:?baseline}" REPS=${REPS:-3} bash tools/legs_ab.sh || exit 1
B="$B" REPS=${REPS:-3} ENVS4=${ENVS4:-131072} bash tools/big_ab.sh
