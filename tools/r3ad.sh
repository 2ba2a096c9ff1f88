# board: the fused rollout's loop-entry wait for the prefetched action (A/B vs without), board tests
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3ad; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_board.py > $O/pytest_board.log 2>&1
rc=$?; tail -2 $O/pytest_board.log; [ $rc -ne 0 ] && { grep -E "^E |FAIL" $O/pytest_board.log | head -20; exit $rc; }
B=boardhead bash tools/board_ab.sh
