#!/bin/bash
# createBoard legs of bench.py (per-step graph + fused rollout), the in-tree library against an
# A/B build (BALLENV_LIB=tools/diag/$B/libballenv.so), interleaved twice.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/board_ab
ARGS="--no-cpu-baseline --steps 10 --warmup 2 --policy-steps 0 --rollout-steps 0 --board-steps 1000 --cold-steps 0 --config2-steps 0 --large-steps 0 --from-reset-steps 0 --blocks-launches 0 --config4-steps 0 --shard-steps 0 --eager-steps 0"
for r in $(seq 1 ${REPS:-2}); do
  for v in new ${B:-boardold}; do   # B: one or more A/B builds under tools/diag
    if [ $v = new ]; then L=""; else L=tools/diag/$v/libballenv.so; fi
    BALLENV_LIB=$L timeout -k 10 200 python3 bench.py $ARGS > gpurun_out/board_ab/$v.$r.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "$v rc=$rc"; tail -5 gpurun_out/board_ab/$v.$r.log; exit $rc; }
    python3 -c "
import json; d = json.loads(open('gpurun_out/board_ab/$v.$r.log').read().strip().splitlines()[-1])['board_profile']
print('%-9s r%s: step %.2f us/step (%.3e env-steps/s), fused %.2f us/step' % ('$v', $r, d['kernel_us_mean'], d['value'], d['fused']['kernel_us_per_step']))"
  done
done
