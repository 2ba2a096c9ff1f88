#!/bin/bash
# createBoard step A/B of library builds: specs "name:lib:ahead" (lib: tools/diag/<lib>/libballenv.so, "-" = in-tree;
# ahead: BALLENV_BOARD_RESET_AHEAD, read by the round-4 reset-ahead builds only), bench.py's board leg (1000 graph-replayed steps + the fused
# rollout), interleaved REPS times.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/board_ahead_ab; mkdir -p $O
ARGS="--no-cpu-baseline --steps 10 --warmup 2 --policy-steps 0 --torch-policy-steps 0 --rollout-steps 0 --board-steps 1000 --cold-steps 0 --config2-steps 0 --config4-steps 0 --large-steps 0 --from-reset-steps 0 --blocks-launches 0"
for r in $(seq 1 ${REPS:-3}); do
  for spec in ${SPECS:-new:-:1 off:-:0}; do
    IFS=: read -r v lib ra <<< "$spec"
    L=""; [ "$lib" != "-" ] && L=tools/diag/$lib/libballenv.so
    BALLENV_LIB=$L BALLENV_BOARD_RESET_AHEAD=$ra timeout -k 10 200 python3 bench.py $ARGS > $O/$v.$r.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "$v rc=$rc"; tail -5 $O/$v.$r.log; exit $rc; }
    python3 -c "
import json; d = json.loads(open('$O/$v.$r.log').read().strip().splitlines()[-1])['board_profile']
print('%-10s r$r: step %.3f us/step (%.3e env-steps/s), fused %.3f us/step' % ('$v', d['kernel_us_mean'], d['value'], d['fused']['kernel_us_per_step']))"
  done
done
