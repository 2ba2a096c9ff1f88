set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_rollout.py tests/test_gpu_episode.py > gpurun_out/r3g_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r3g_pytest.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error" gpurun_out/r3g_pytest.log | head; exit $rc; }
timeout -k 10 400 python tools/lane_sweep.py --rollout --window 5 --envs 4096,8192,16384,32768,65536 --lanes 1,4,8 --steps 1000 > gpurun_out/r3g_sweep_roll5.jsonl 2> gpurun_out/r3g_sweep_roll5.err
rc=$?; cat gpurun_out/r3g_sweep_roll5.jsonl; [ $rc -ne 0 ] && { tail -20 gpurun_out/r3g_sweep_roll5.err; exit $rc; }
