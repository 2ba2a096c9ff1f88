set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
BALLENV_LIB=tools/diag/st/libballenv.so timeout -k 10 200 python tools/board_phases.py > gpurun_out/r3o_board_phases.txt 2>&1
rc=$?; cat gpurun_out/r3o_board_phases.txt; exit $rc
