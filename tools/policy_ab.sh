#!/bin/bash
# Config-5 fused policy rollout (bench.py's policy_rollout line), the in-tree library against an
# A/B build (BALLENV_LIB=tools/diag/$B/libballenv.so), interleaved twice.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pol_ab
ARGS="--no-cpu-baseline --steps 10 --warmup 2 --policy-steps 1000 --torch-policy-steps 0 --board-steps 0 --rollout-steps 0 --cold-steps 0 --config2-steps 0 --large-steps 0 --from-reset-steps 0 --blocks-launches 0"
for r in 1 2; do
  for v in new ${B:-rohead}; do   # B: one or more A/B builds
    if [ $v = new ]; then L=""; else L=tools/diag/$v/libballenv.so; fi
    BALLENV_LIB=$L timeout -k 10 200 python3 bench.py $ARGS > gpurun_out/pol_ab/$v.$r.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "$v rc=$rc"; tail -5 gpurun_out/pol_ab/$v.$r.log; exit $rc; }
    python3 -c "
import json; d = json.loads(open('gpurun_out/pol_ab/$v.$r.log').read().strip().splitlines()[-1])['policy_rollout']
print('%-7s r%s: fused policy rollout %.3f us/step (%.3e env-steps/s), two-launch policy_kernel %.2f us' % ('$v', $r, d['kernel_us_per_step'], d['value'], d['two_launch']['policy_kernel_us']))"
  done
done
