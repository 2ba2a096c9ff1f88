#!/bin/bash
# A/B of library builds on the step, fused-rollout and fused-policy legs: args "name@lib" (lib empty:
# the in-tree build).  One bench.py run each (1000 steps per leg, no CPU baseline / board / torch legs).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/legs
for spec in "$@"; do
  n=${spec%%@*}; l=${spec#*@}
  BALLENV_LIB=$l timeout -k 10 150 python3 bench.py --no-cpu-baseline --steps 1000 --warmup 100 --policy-steps 1000 \
      --torch-policy-steps 0 --board-steps 0 --rollout-steps 1000 --cold-steps 0 --config2-steps 0 --large-steps 0 --from-reset-steps 0 --blocks-launches 0 > gpurun_out/legs/$n.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "$n rc=$rc"; tail -5 gpurun_out/legs/$n.log; exit $rc; }
  python3 -c "
import json; d = json.loads(open('gpurun_out/legs/$n.log').read().strip().splitlines()[-1])
print('%-10s step %.3f  fused %.3f  policy %.3f' % ('$n', d['roofline']['kernel_us_mean'], d['fused_rollout']['kernel_us_per_step'], d['policy_rollout']['kernel_us_per_step']))"
done
