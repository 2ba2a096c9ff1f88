#!/bin/bash
# Batch-size sweep of the step API headline leg (and the fused random-action rollout): one bench.py
# run per size, legs off except the rollout; JSON lines to gpurun_out/sweep.jsonl.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; : > gpurun_out/sweep.jsonl
for spec in ${SIZES:-4096:5 65536:10 262144:10 1048576:10}; do   # envs:window
  set -- ${spec/:/ }
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --envs $1 --window $2 --steps 1000 --warmup 100 --policy-steps 0 \
      --board-steps 0 --rollout-steps 1000 > gpurun_out/sweep_$1.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "envs $1 rc=$rc"; tail -5 gpurun_out/sweep_$1.log; exit $rc; }
  tail -1 gpurun_out/sweep_$1.log >> gpurun_out/sweep.jsonl
  python3 -c "
import json; d = json.loads(open('gpurun_out/sweep_$1.log').read().strip().splitlines()[-1]); r = d['roofline']; f = d['fused_rollout']
print('envs %8d W=%-2d step %.3e env-steps/s kernel %.2f us frac %.3f (engine %.3f) | fused %.3e (%.2f us)' % ($1, $2, d['value'], r['kernel_us_mean'], r['frac'], r['engine_frac'], f['value'], f['kernel_us_per_step']))"
done
