set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python tools/lane_sweep.py --window 5 --envs 4096 --lanes 1,8,4 --reps 3 > gpurun_out/r3e_sweep5.jsonl 2> gpurun_out/r3e_sweep5.err
rc=$?; cat gpurun_out/r3e_sweep5.jsonl; [ $rc -ne 0 ] && { tail -20 gpurun_out/r3e_sweep5.err; exit $rc; }
BALLENV_LIB=tools/diag/skip/libballenv.so W=5 SIZES=4096 GRAPH=1 MASKS=0,256,4,1,5,16384 \
  timeout -k 10 240 python tools/ablate.py > gpurun_out/r3e_ablate5.jsonl 2> gpurun_out/r3e_ablate5.err
rc=$?; cat gpurun_out/r3e_ablate5.jsonl; [ $rc -ne 0 ] && { tail -20 gpurun_out/r3e_ablate5.err; exit $rc; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_episode.py > gpurun_out/r3e_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r3e_pytest.log; exit $rc
