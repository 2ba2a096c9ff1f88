# Policy / rollout GPU tests, then the config-5 (tools/policy_ab.sh) and random-action fused
# rollout (tools/rollout_ab.sh) A/Bs of the in-tree library against tools/diag/$B.
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/pol
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "policy or rollout" > gpurun_out/pol/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/pol/pytest.log; [ $rc -ne 0 ] && exit $rc
B="${B:-old}" timeout -k 10 900 bash tools/policy_ab.sh || exit $?
[ "${RO:-1}" = 1 ] && B="${B:-old}" timeout -k 10 900 bash tools/rollout_ab.sh
