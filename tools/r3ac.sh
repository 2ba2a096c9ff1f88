# board: loop-entry wait of the prefetched action, 16-B sc1 agent/goal stores, static-only reset rounds: tests, A/B, phases, counters
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3ac; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_board.py > $O/pytest_board.log 2>&1
rc=$?; tail -2 $O/pytest_board.log; [ $rc -ne 0 ] && { grep -E "^E |FAIL" $O/pytest_board.log | head -20; exit $rc; }
B="boardnorounds boardbase" bash tools/board_ab.sh || exit 1
BALLENV_LIB=tools/diag/st/libballenv.so timeout -k 10 200 python tools/board_phases.py 2>&1 | grep -v amdgpu.ids
PASSES="FETCH_SIZE WRITE_SIZE" timeout -k 10 600 bash tools/pmc_passes.sh r3ac/pmc --no-cpu-baseline --steps 10 --warmup 2 --settle 10 \
    --policy-steps 0 --torch-policy-steps 0 --board-steps 200 --rollout-steps 0 --cold-steps 0 \
    --config2-steps 0 --large-steps 0 --from-reset-steps 0 --blocks-launches 0
python tools/pmc_report.py $O/pmc "board_kernel<6, false" 65536 | grep -o '"hbm_bytes_per_unit": [0-9.]*'
