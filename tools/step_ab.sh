#!/bin/bash
# Step API headline and cold_action_rows lines, the in-tree library against an A/B build
# (BALLENV_LIB=tools/diag/$B/libballenv.so), interleaved twice.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/step_ab
ARGS="--no-cpu-baseline --policy-steps 0 --board-steps 0 --rollout-steps 0"
for r in 1 2; do
  for v in new ${B:-alast}; do
    if [ $v = new ]; then L=""; else L=tools/diag/$v/libballenv.so; fi
    BALLENV_LIB=$L timeout -k 10 200 python3 bench.py $ARGS > gpurun_out/step_ab/$v.$r.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "$v rc=$rc"; tail -5 gpurun_out/step_ab/$v.$r.log; exit $rc; }
    python3 -c "
import json; d = json.loads([l for l in open('gpurun_out/step_ab/$v.$r.log') if l.startswith('{')][-1]); c = d['cold_action_rows']
print('%-6s r%s: step %.3f us (%.3e) | cold rows %.3f us (%.3e)' % ('$v', $r, d['roofline']['kernel_us_mean'], d['value'], c['kernel_us_mean'], c['value']))"
  done
done
