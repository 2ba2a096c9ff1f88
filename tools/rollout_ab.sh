#!/bin/bash
# Fused random-action rollout (bench.py's fused_rollout line) and the step API, the in-tree
# library against an A/B build (BALLENV_LIB=tools/diag/$B/libballenv.so), interleaved twice.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ro_ab
ARGS="--no-cpu-baseline --steps 1000 --warmup 50 --policy-steps 0 --board-steps 0 --rollout-steps 2000 --cold-steps 0 --config2-steps 0 --large-steps 0 --from-reset-steps 0 --blocks-launches 0"
for r in 1 2; do
  for v in new ${B:-rohead}; do
    if [ $v = new ]; then L=""; else L=tools/diag/$v/libballenv.so; fi
    BALLENV_LIB=$L timeout -k 10 200 python3 bench.py $ARGS > gpurun_out/ro_ab/$v.$r.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "$v rc=$rc"; tail -5 gpurun_out/ro_ab/$v.$r.log; exit $rc; }
    python3 -c "
import json; d = json.loads(open('gpurun_out/ro_ab/$v.$r.log').read().strip().splitlines()[-1]); f = d['fused_rollout']
print('%-7s r%s: step %.3f us, fused rollout %.3f us/step (%.3e env-steps/s)' % ('$v', $r, d['roofline']['kernel_us_mean'], f['kernel_us_per_step'], f['value']))"
  done
done
