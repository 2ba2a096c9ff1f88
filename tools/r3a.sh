set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_bench_contract.py "tests/test_gpu_rollout.py::test_fused_rollouts_non_default_radius" "tests/test_gpu_episode.py::test_step2_equals_one_lane_kernel" > gpurun_out/r3a_pytest.log 2>&1
rc=$?; tail -5 gpurun_out/r3a_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3a_bench.log 2>&1
rc=$?; tail -c 3000 gpurun_out/r3a_bench.log; exit $rc
