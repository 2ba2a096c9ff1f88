cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_rollout.py tests/test_gpu_policy.py -x -q --timeout 200 --timeout-method thread > gpurun_out/roll_test.log 2>&1; rc=$?; tail -3 gpurun_out/roll_test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/fused_ablate.py 0 > gpurun_out/abl_prod.log 2>&1 || exit $?
timeout -k 10 300 python tools/policy_ablate.py 0 > gpurun_out/pabl.log 2>&1 || exit $?
grep -h "dbg=" gpurun_out/abl_prod.log gpurun_out/pabl.log
