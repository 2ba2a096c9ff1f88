set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_rollout.py tests/test_gpu_episode.py > gpurun_out/r3j_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r3j_pytest.log; [ $rc -ne 0 ] && { grep -E "^E " gpurun_out/r3j_pytest.log | head; exit $rc; }
bash tools/ab_legs.sh new@ old@tools/diag/oldpol/libballenv.so new2@ old2@tools/diag/oldpol/libballenv.so
