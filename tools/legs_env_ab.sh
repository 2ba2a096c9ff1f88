#!/bin/bash
# Like legs_ab.sh, with "name:lib:VAR=val" specs (lib empty: the in-tree build; VAR=val optional):
# the headline step, config 2 and config 4 at ENVS4 on one rank, interleaved REPS times.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/legs_env_ab; mkdir -p $O
ARGS="--no-cpu-baseline --steps 1000 --warmup 100 --policy-steps 0 --torch-policy-steps 0 --board-steps 0 --rollout-steps 0 --cold-steps 0 --config2-steps 1000 --config4-steps 1000 --config4-envs ${ENVS4:-32768} --large-steps 0 --from-reset-steps 0 --blocks-launches 0 --shard-steps 0 --eager-steps 0"
for r in $(seq 1 ${REPS:-2}); do
  for spec in ${SPECS}; do
    IFS=: read -r n l ev <<< "$spec"
    env ${ev:+$ev} BALLENV_LIB=$l timeout -k 10 200 python3 bench.py $ARGS > $O/$n.$r.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "$n rc=$rc"; tail -5 $O/$n.$r.log; exit $rc; }
    python3 -c "
import json; d = json.loads(open('$O/$n.$r.log').read().strip().splitlines()[-1])
print('%-8s r$r: step %.3f  config2 %.3f  config4@%d %.3f us' % ('$n', d['roofline']['kernel_us_mean'], d['config2']['kernel_us_mean'], d['config4']['envs_per_rank'], d['config4']['kernel_us_mean']))"
  done
done
