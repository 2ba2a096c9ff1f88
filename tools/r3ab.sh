# policy image / obs-row staging with 8 loads in flight: policy + rollout GPU tests, config-5 A/B;
# blocks chunk-size A/B
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r3ab
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_policy.py tests/test_gpu_rollout.py tests/test_gpu_episode.py -m gpu -k "policy or rollout" > gpurun_out/r3ab/pytest_pol.log 2>&1
rc=$?; tail -2 gpurun_out/r3ab/pytest_pol.log; [ $rc -ne 0 ] && { grep -E "^E |FAIL" gpurun_out/r3ab/pytest_pol.log | head -20; exit $rc; }
B=polold bash tools/policy_ab.sh || exit 1
B="featch6 featold" bash tools/blocks_ab.sh || exit 1
# board: action table in LDS + the fused rollout's next action read one step ahead
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_board.py > gpurun_out/r3ab/pytest_board.log 2>&1
rc=$?; tail -2 gpurun_out/r3ab/pytest_board.log; [ $rc -ne 0 ] && { grep -E "^E |FAIL" gpurun_out/r3ab/pytest_board.log | head -20; exit $rc; }
B=boardpf0 bash tools/board_ab.sh
BALLENV_LIB=tools/diag/st/libballenv.so timeout -k 10 200 python tools/board_phases.py 2>&1 | grep -v amdgpu.ids
