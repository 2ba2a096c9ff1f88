set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python tools/lane_sweep.py --window 5 --envs 4096,8192,16384,32768,65536 --lanes 1,4,8 > gpurun_out/r3b_sweep5.jsonl 2> gpurun_out/r3b_sweep5.err
rc=$?; cat gpurun_out/r3b_sweep5.jsonl; [ $rc -ne 0 ] && { tail -20 gpurun_out/r3b_sweep5.err; exit $rc; }
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_episode.py tests/test_bench_contract.py "tests/test_gpu_rollout.py::test_fused_rollouts_non_default_radius" "tests/test_gpu_parity.py::test_save_load_state_blob_round_trip" > gpurun_out/r3b_pytest.log 2>&1
rc=$?; tail -8 gpurun_out/r3b_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3b_bench.log 2>&1
rc=$?; tail -c 4000 gpurun_out/r3b_bench.log; exit $rc
