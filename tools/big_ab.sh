#!/bin/bash
# A/B of library builds on the one-lane fixed step kernel's legs: config 4 on one rank (262 144 envs)
# and the 2^20-env large batch, 1000 graph-replayed steps each, interleaved REPS times.
# B="name ..." -> tools/diag/name/libballenv.so; "new" = in-tree.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/big_ab; mkdir -p $O
ARGS="--no-cpu-baseline --steps 10 --warmup 2 --policy-steps 0 --torch-policy-steps 0 --board-steps 0 --rollout-steps 0 --cold-steps 0 --config2-steps 0 --config4-steps 1000 --config4-envs ${ENVS4:-262144} --large-steps ${LARGE:-1000} --from-reset-steps 0 --blocks-launches 0 --shard-steps 0 --eager-steps 0"
for r in $(seq 1 ${REPS:-3}); do
  for v in new ${B}; do
    L=""; [ $v != new ] && L=tools/diag/$v/libballenv.so
    BALLENV_LIB=$L timeout -k 10 200 python3 bench.py $ARGS > $O/$v.$r.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "$v rc=$rc"; tail -5 $O/$v.$r.log; exit $rc; }
    python3 -c "
import json; d = json.loads(open('$O/$v.$r.log').read().strip().splitlines()[-1])
print('%-6s r$r: config4@%d %.3f us  large(2^20) %s' % ('$v', d['config4']['envs_per_rank'], d['config4']['kernel_us_mean'], d['large_batch']['kernel_us_mean'] if d.get('large_batch') else '-'))"
  done
done
