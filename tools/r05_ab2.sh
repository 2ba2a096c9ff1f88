#!/bin/bash
# Round 5, second A/B session: step2_kernel prologue variants (BE_S2_PRO 1 = in-tree, 2, 3; base =
# the pre-fix library, i.e. variant 0), the createBoard prologue (per-step and fused), the reset
# pass's cost, phase stamps and the kernarg-preload probe.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05_c; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_board.py tests/test_gpu_episode.py -m gpu -x -q -p no:cacheprovider --timeout 150 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
B="base s2p2 s2p3" REPS=3 bash tools/legs_ab.sh || exit 1
B=base REPS=3 bash tools/board_ab.sh || exit 1
timeout -k 10 200 python tools/reset_cost.py > $O/reset_cost.txt 2>&1 || { tail -5 $O/reset_cost.txt; exit 1; }
cat $O/reset_cost.txt
bash tools/probe/preload_probe.sh > $O/preload_probe.txt 2>&1 || { tail -5 $O/preload_probe.txt; exit 1; }
cat $O/preload_probe.txt
for n in 32768 65536; do
  BALLENV_STEP_LPE=2 timeout -k 10 120 ./tools/stamps $n > $O/stamps_step2_$n.txt 2>&1 || { tail -5 $O/stamps_step2_$n.txt; exit 1; }
done
echo done
