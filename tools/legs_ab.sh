#!/bin/bash
# Step-API legs per library build, interleaved REPS times: the headline step (65 536 envs, W=10),
# config 2 (4 096, W=5) and config 4 at ENVS4 global envs on one rank (default 32 768: the N=8
# shard), 1000 graph-replayed steps each.  B="name ..." -> tools/diag/name/libballenv.so; "new" = in-tree.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/legs_ab; mkdir -p $O
ARGS="--no-cpu-baseline --steps 1000 --warmup 100 --policy-steps 0 --torch-policy-steps 0 --board-steps 0 --rollout-steps 0 --cold-steps 0 --config2-steps 1000 --config4-steps 1000 --config4-envs ${ENVS4:-32768} --large-steps 0 --from-reset-steps 0 --blocks-launches 0 --shard-steps 0 --eager-steps 0"
for r in $(seq 1 ${REPS:-2}); do
  for v in new ${B}; do
    L=""; [ $v != new ] && L=tools/diag/$v/libballenv.so
    BALLENV_LIB=$L timeout -k 10 200 python3 bench.py $ARGS > $O/$v.$r.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "$v rc=$rc"; tail -5 $O/$v.$r.log; exit $rc; }
    python3 -c "
import json; d = json.loads(open('$O/$v.$r.log').read().strip().splitlines()[-1])
print('%-8s r$r: step %.3f  config2 %.3f  config4@%d %.3f us' % ('$v', d['roofline']['kernel_us_mean'], d['config2']['kernel_us_mean'], d['config4']['envs_per_rank'], d['config4']['kernel_us_mean']))"
  done
done
