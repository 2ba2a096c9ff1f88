set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
# 1) stepw phase ablation at config 2 (diagnostics build), graph-replayed launches
BALLENV_LIB=tools/diag/skip/libballenv.so W=5 SIZES=4096 GRAPH=1 MASKS=0,64,128,1152,256,4,16384,1,8,5 \
  timeout -k 10 240 python tools/ablate.py > gpurun_out/r3c_ablate5.jsonl 2> gpurun_out/r3c_ablate5.err
rc=$?; cat gpurun_out/r3c_ablate5.jsonl; [ $rc -ne 0 ] && { tail -20 gpurun_out/r3c_ablate5.err; exit $rc; }
BALLENV_LIB=tools/diag/skip/libballenv.so BALLENV_STEP5_LPE=1 W=5 SIZES=4096 GRAPH=1 MASKS=0,64,128,256,4 \
  timeout -k 10 240 python tools/ablate.py > gpurun_out/r3c_ablate5_lpe1.jsonl 2>> gpurun_out/r3c_ablate5.err
rc=$?; cat gpurun_out/r3c_ablate5_lpe1.jsonl; [ $rc -ne 0 ] && exit $rc
# 2) prev_dist read vs recompute (A/B in one process): W=10 headline, W=5 config 2
timeout -k 10 240 python tools/lane_sweep.py --window 10 --envs 65536 --var BALLENV_PREV_READ --lanes 1,0 --reps 3 > gpurun_out/r3c_prevread.jsonl 2> gpurun_out/r3c_prevread.err
rc=$?; cat gpurun_out/r3c_prevread.jsonl; [ $rc -ne 0 ] && { tail -20 gpurun_out/r3c_prevread.err; exit $rc; }
timeout -k 10 240 python tools/lane_sweep.py --window 5 --envs 4096 --var BALLENV_PREV_READ --lanes 1,0 --reps 3 >> gpurun_out/r3c_prevread.jsonl 2>> gpurun_out/r3c_prevread.err
rc=$?; tail -6 gpurun_out/r3c_prevread.jsonl; [ $rc -ne 0 ] && exit $rc
# 3) tests touched since the last run
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_board.py tests/test_gpu_episode.py tests/test_gpu_parity.py > gpurun_out/r3c_pytest.log 2>&1
rc=$?; tail -5 gpurun_out/r3c_pytest.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error" gpurun_out/r3c_pytest.log | head; exit $rc; }
# 4) board legs (two lanes vs one)
for l in 2 1; do
  BALLENV_BOARD_LPE=$l timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 5 --policy-steps 0 --rollout-steps 0 --cold-steps 0 --config2-steps 0 --large-steps 0 --from-reset-steps 0 > gpurun_out/r3c_board_lpe$l.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { tail -5 gpurun_out/r3c_board_lpe$l.log; exit $rc; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/r3c_board_lpe$l.log').read().splitlines()[-1])['board_profile']; print('board lpe$l', d['kernel_us_mean'], d['fused']['kernel_us_per_step'])"
done
