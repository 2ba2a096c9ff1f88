#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05_e; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_episode.py tests/test_gpu_graph.py tests/test_gpu_rollout.py -m gpu -x -q -p no:cacheprovider --timeout 150 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
SPECS="base:tools/diag/base/libballenv.so: new:: off::BALLENV_EARLY_RESET=0" REPS=3 bash tools/legs_env_ab.sh || exit 1
timeout -k 10 200 python tools/reset_cost.py > $O/reset_cost.txt 2>&1 || { tail -5 $O/reset_cost.txt; exit 1; }
cat $O/reset_cost.txt
