set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python tools/lane_sweep.py --window 5 --envs 4096,8192,16384 --lanes 1,4,8 > gpurun_out/r3d_sweep5.jsonl 2> gpurun_out/r3d_sweep5.err
rc=$?; cat gpurun_out/r3d_sweep5.jsonl; [ $rc -ne 0 ] && { tail -20 gpurun_out/r3d_sweep5.err; exit $rc; }
BALLENV_LIB=tools/diag/skip/libballenv.so W=5 SIZES=4096 GRAPH=1 MASKS=0,256,4,1,5,16384 \
  timeout -k 10 240 python tools/ablate.py > gpurun_out/r3d_ablate5.jsonl 2> gpurun_out/r3d_ablate5.err
rc=$?; cat gpurun_out/r3d_ablate5.jsonl; [ $rc -ne 0 ] && { tail -20 gpurun_out/r3d_ablate5.err; exit $rc; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_episode.py tests/test_board.py > gpurun_out/r3d_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r3d_pytest.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error" gpurun_out/r3d_pytest.log | head; exit $rc; }
# PMC passes on the config-2 (200 steps) and large-batch (100 timed steps) legs
bash tools/pmc_passes.sh r3d_pmc --no-cpu-baseline --steps 10 --warmup 2 --settle 10 --policy-steps 0 --board-steps 0 \
  --rollout-steps 0 --cold-steps 0 --from-reset-steps 0 --config2-steps 200 --large-steps 100 > gpurun_out/r3d_pmc.log 2>&1
rc=$?; cat gpurun_out/r3d_pmc.log; [ $rc -ne 0 ] && exit $rc
python tools/pmc_report.py gpurun_out/r3d_pmc "stepw_kernel<5, 13, 5, 8>" 4096 --out gpurun_out/r3d_pmc_config2.json > /dev/null && \
python tools/pmc_report.py gpurun_out/r3d_pmc "be_kernel<10, 0, 13, 5>" 1048576 --out gpurun_out/r3d_pmc_large.json > /dev/null
rc=$?; python -c "
import json
for f in ('gpurun_out/r3d_pmc_config2.json','gpurun_out/r3d_pmc_large.json'):
    d=json.load(open(f)); print(f, d['kernel'], d.get('hbm_bytes_per_unit'), d.get('dispatches'), d.get('per_wave'), d.get('wave_cycle_split'))
"
exit $rc
