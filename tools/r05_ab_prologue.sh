#!/bin/bash
# Round 5: the prologue fix (every load issued before the first wait) -- parity tests of the step
# kernels, interleaved A/B against the HEAD library (tools/diag/base), the eager step() host cost
# against round 4's batched.py, the reset pass's cost (tools/reset_cost.py) and phase stamps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05_b; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_episode.py tests/test_gpu_graph.py tests/test_gpu_coord_range.py tests/test_board.py -m gpu -x -q -p no:cacheprovider --timeout 150 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
B=base REPS=3 bash tools/legs_ab.sh || exit 1
ENVS4=131072 B=base REPS=2 bash tools/legs_ab.sh || exit 1
B=base REPS=3 bash tools/board_ab.sh || exit 1
timeout -k 10 200 python tools/eager_ab.py > $O/eager_ab.txt 2>&1 || { tail -5 $O/eager_ab.txt; exit 1; }
cat $O/eager_ab.txt
timeout -k 10 200 python tools/reset_cost.py > $O/reset_cost.txt 2>&1 || { tail -5 $O/reset_cost.txt; exit 1; }
cat $O/reset_cost.txt
for n in 32768 65536; do
  BALLENV_STEP_LPE=2 timeout -k 10 120 ./tools/stamps $n > $O/stamps_step2_$n.txt 2>&1 || { tail -5 $O/stamps_step2_$n.txt; exit 1; }
done

bash tools/probe/preload_probe.sh > gpurun_out/r05_b/preload_probe.txt 2>&1; cat gpurun_out/r05_b/preload_probe.txt
echo done
