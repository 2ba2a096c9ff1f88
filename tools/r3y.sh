# board: write-through stores (tests, A/B vs the previous library and vs sc1 in the fused rollout too);
# prep_state2 blocks: batched obstacle loads + sc1 copy-out (tests, A/B vs the previous features.hip)
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r3y
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_board.py > gpurun_out/r3y/pytest_board.log 2>&1
rc=$?; tail -2 gpurun_out/r3y/pytest_board.log; [ $rc -ne 0 ] && { grep -E "^E |FAIL" gpurun_out/r3y/pytest_board.log | head -20; exit $rc; }
B="boardprev boardwtroll" bash tools/board_ab.sh || exit 1
B=featold bash tools/blocks_ab.sh
