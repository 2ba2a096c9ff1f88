#!/bin/bash
# BASELINE config 2 (4 096 envs, W=5, stepw_kernel): bench.py's config2 leg, the in-tree library
# against tools/diag/$B, interleaved twice (1 000 graph-replayed steps each).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/c2_ab; mkdir -p $O
ARGS="--no-cpu-baseline --steps 10 --warmup 2 --settle 10 --policy-steps 0 --torch-policy-steps 0 --board-steps 0 --rollout-steps 0 --cold-steps 0 --config2-steps 1000 --large-steps 0 --from-reset-steps 0 --blocks-launches 0"
for r in $(seq 1 ${REPS:-2}); do
  for v in new ${B:-stepwold}; do
    if [ $v = new ]; then L=""; else L=tools/diag/$v/libballenv.so; fi
    BALLENV_LIB=$L timeout -k 10 200 python3 bench.py $ARGS > $O/$v.$r.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "$v rc=$rc"; tail -5 $O/$v.$r.log; exit $rc; }
    python3 -c "
import json; d = json.loads(open('$O/$v.$r.log').read().strip().splitlines()[-1])['config2']
print('%-9s r$r: config2 %.3f us/step (%.3e env-steps/s), %s' % ('$v', d['kernel_us_mean'], d['value'], d['kernel']))"
  done
done
