# stepw prologue (all loads issued before the first wait): stepw / config-2 GPU tests + A/B; blocks tests + A/B
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r3z
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_episode.py tests/test_gpu_rollout.py -m gpu -k "stepw or 5-4096 or goal_change or rolloutw" > gpurun_out/r3z/pytest_stepw.log 2>&1
rc=$?; tail -2 gpurun_out/r3z/pytest_stepw.log; [ $rc -ne 0 ] && { grep -E "^E |FAIL" gpurun_out/r3z/pytest_stepw.log | head -20; exit $rc; }
bash tools/c2_ab.sh || exit 1
B=featold bash tools/blocks_ab.sh
