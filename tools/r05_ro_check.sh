#!/bin/bash
# Fused-rollout tests, then tools/r05_ro_ab.sh against tools/diag/$B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp; O=gpurun_out/r05_ro; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_rollout.py tests/test_gpu_policy.py tests/test_gpu_episode.py -m gpu -x -q -p no:cacheprovider --timeout 150 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/r05_ro_ab.sh
