set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
BALLENV_LIB=tools/diag/st/libballenv.so timeout -k 10 200 python tools/rolloutw_phases.py > gpurun_out/r3i_phases.txt 2>&1
rc=$?; head -10 gpurun_out/r3i_phases.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_rollout.py -k "rolloutw or default" > gpurun_out/r3i_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r3i_pytest.log; [ $rc -ne 0 ] && { grep -E "^E " gpurun_out/r3i_pytest.log | head; exit $rc; }
timeout -k 10 300 python tools/lane_sweep.py --rollout --window 5 --envs 4096,16384 --lanes 1,8 --steps 1000 > gpurun_out/r3i_sweep.jsonl 2> gpurun_out/r3i_sweep.err
rc=$?; cat gpurun_out/r3i_sweep.jsonl; exit $rc
