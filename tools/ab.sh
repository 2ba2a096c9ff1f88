#!/bin/bash
# Interleaved A/B of ARMS on the step-API legs: the headline step (65 536 envs, W=10), config 2
# (4 096, W=5) and config 4 at ENVS4 global envs on one rank (default 32 768: the N=8 shard), 1 000
# graph-replayed steps each, REPS rounds, arms in turn within a round.  An arm is a name; its
# library is LIB_<name> (default: the in-tree one) and its environment ENV_<name> (space-separated
# VAR=value, e.g. BALLENV_POOL=0).  Replaces round 5's one-off tools/r05_ab*.sh drivers.
#   ARMS="pool nopool" ENV_nopool="BALLENV_POOL=0" REPS=3 bash tools/ab.sh
#   ARMS="new r05" LIB_r05=tools/diag/r05/libballenv.so bash tools/ab.sh
# EXTRA: more bench.py arguments (e.g. "--rollout-steps 1000" to add the fused legs).
# LEG=board: the createBoard leg instead (65 536 envs, 1 000 graph-replayed be_board_step calls and
# the same steps fused, 100 per launch), with the headline leg cut to 50 steps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-ab}; mkdir -p $O
if [ "${LEG:-step}" = board ]; then
  ARGS="--no-cpu-baseline --steps 50 --warmup 10 --policy-steps 0 --torch-policy-steps 0 --board-steps 1000 --rollout-steps 0 --cold-steps 0 --config2-steps 0 --config4-steps 0 --large-steps 0 --from-reset-steps 0 --blocks-launches 0 --shard-steps 0 --eager-steps 0 ${EXTRA:-}"
else
  ARGS="--no-cpu-baseline --steps 1000 --warmup 100 --policy-steps 0 --torch-policy-steps 0 --board-steps 0 --rollout-steps 0 --cold-steps 0 --config2-steps 1000 --config4-steps 1000 --config4-envs ${ENVS4:-32768} --large-steps 0 --from-reset-steps 0 --blocks-launches 0 --shard-steps 0 --eager-steps 0 ${EXTRA:-}"
fi
for r in $(seq 1 ${REPS:-3}); do
  for v in ${ARMS:?ARMS}; do
    lv=LIB_$v; ev=ENV_$v
    env ${!ev:-} BALLENV_LIB=${!lv:-} timeout -k 10 200 python3 bench.py $ARGS > $O/$v.$r.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "$v rc=$rc"; tail -5 $O/$v.$r.log; exit $rc; }
    python3 -c "
import json; d = json.loads(open('$O/$v.$r.log').read().strip().splitlines()[-1])
bp = d.get('board_profile')
if bp:
    print('%-8s r$r: board step %.3f  fused %.3f us' % ('$v', bp['kernel_us_mean'], bp['fused']['kernel_us_per_step']), flush=True)
    raise SystemExit
s = '%-8s r$r: step %.3f  config2 %.3f  config4@%d %.3f us' % ('$v', d['roofline']['kernel_us_mean'], d['config2']['kernel_us_mean'], d['config4']['envs_per_rank'], d['config4']['kernel_us_mean'])
if d.get('large_batch'): s += '  large %.3f' % d['large_batch']['kernel_us_mean']
if d.get('fused_rollout'): s += '  fused %.3f' % d['fused_rollout']['kernel_us_per_step']
if d.get('policy_rollout'): s += '  policy %.3f' % d['policy_rollout']['kernel_us_per_step']
print(s, flush=True)"
  done
done
