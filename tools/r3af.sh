# fused rollouts: the episode return lands before the step loop (no per-step vmcnt(0)): rollout
# tests, A/B of the step / fused / policy legs against the build without it
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3af; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_rollout.py tests/test_gpu_episode.py -m gpu > $O/pytest_rollout.log 2>&1
rc=$?; tail -2 $O/pytest_rollout.log; [ $rc -ne 0 ] && { grep -E "^E |FAIL" $O/pytest_rollout.log | head -20; exit $rc; }
bash tools/ab_legs.sh new@ noret@tools/diag/noret/libballenv.so new2@ noret2@tools/diag/noret/libballenv.so
