set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r3x
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_board.py > gpurun_out/r3x/pytest_board.log 2>&1
rc=$?; tail -2 gpurun_out/r3x/pytest_board.log; [ $rc -ne 0 ] && { grep -E "^E |FAIL" gpurun_out/r3x/pytest_board.log | head -20; exit $rc; }
BALLENV_LIB=tools/diag/st/libballenv.so timeout -k 10 200 python tools/board_phases.py 2>&1 | grep -v amdgpu.ids
B="boardprev boardwtroll" bash tools/board_ab.sh
