set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_policy.py tests/test_gpu_rollout.py "tests/test_gpu_episode.py::test_policy_rollout_default_episode" > gpurun_out/r3f_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r3f_pytest.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error" gpurun_out/r3f_pytest.log | head; exit $rc; }
B=oldpol bash tools/policy_ab.sh
