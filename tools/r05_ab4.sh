#!/bin/bash
# Round 5: step2_kernel's early truncation reset (the pair's odd lanes draw the reset blocks) --
# parity tests of the step kernels, then an interleaved A/B against the pre-round library (base)
# and the reset-cost arms (tools/reset_cost.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05_d; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_episode.py tests/test_gpu_graph.py tests/test_gpu_rollout.py tests/test_gpu_parity.py tests/test_gpu_coord_range.py tests/test_gpu_dist.py -m gpu -x -q -p no:cacheprovider --timeout 150 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
B="base" REPS=3 bash tools/legs_ab.sh || exit 1
timeout -k 10 200 python tools/reset_cost.py > $O/reset_cost.txt 2>&1 || { tail -5 $O/reset_cost.txt; exit 1; }
cat $O/reset_cost.txt
echo done
