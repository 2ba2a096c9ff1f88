#!/bin/bash
# Fused rollouts (random-action be_rollout and config-5 be_policy_rollout) of the in-tree library against
# tools/diag/$B, interleaved REPS times.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/ro_ab5; mkdir -p $O
ARGS="--no-cpu-baseline --steps 100 --warmup 10 --policy-steps ${PSTEPS:-1000} --torch-policy-steps 0 --board-steps 0 --rollout-steps 2000 --cold-steps 0 --config2-steps 0 --config4-steps 0 --large-steps 0 --from-reset-steps 0 --blocks-launches 0 --shard-steps 0 --eager-steps 0"
for r in $(seq 1 ${REPS:-3}); do
  for v in new ${B:?baseline}; do
    L=""; [ $v != new ] && L=tools/diag/$v/libballenv.so
    BALLENV_LIB=$L timeout -k 10 300 python3 bench.py $ARGS > $O/$v.$r.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "$v rc=$rc"; tail -5 $O/$v.$r.log; exit $rc; }
    python3 -c "
import json; d = json.loads(open('$O/$v.$r.log').read().strip().splitlines()[-1]); f = d['fused_rollout']; q = d.get('policy_rollout') or {}
print('%-5s r$r: fused rollout %.3f us/step  policy rollout %s us/step' % ('$v', f['kernel_us_per_step'], q.get('kernel_us_per_step')))"
  done
done
