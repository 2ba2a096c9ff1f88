#!/bin/bash
# Interleaved A/B of library builds (tools/diag/NAME/libballenv.so; "new" = in-tree) on the
# config-2, createBoard, headline-step, fused-rollout and fused-policy legs of bench.py.
# usage: B="r3end pre_dde" REPS=2 bash tools/rev_ab.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/rev_ab; mkdir -p $O
ARGS="--no-cpu-baseline --steps 1000 --warmup 100 --policy-steps 1000 --torch-policy-steps 0 --board-steps 1000 \
  --rollout-steps 1000 --cold-steps 0 --config2-steps 1000 --config4-steps 0 --large-steps 0 --from-reset-steps 0 --blocks-launches 0"
for r in $(seq 1 ${REPS:-2}); do
  for v in new ${B}; do
    if [ $v = new ]; then L=""; else L=tools/diag/$v/libballenv.so; fi
    BALLENV_LIB=$L timeout -k 10 200 python3 bench.py $ARGS > $O/$v.$r.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "$v rc=$rc"; tail -5 $O/$v.$r.log; exit $rc; }
    python3 - $O/$v.$r.log $v $r <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("%-8s r%s  step %.3f  c2 %.3f  board %.3f/%.3f  fused %.3f  policy %.3f" % (sys.argv[2], sys.argv[3],
      d["roofline"]["kernel_us_mean"], d["config2"]["kernel_us_mean"], d["board_profile"]["kernel_us_mean"],
      d["board_profile"]["fused"]["kernel_us_per_step"], d["fused_rollout"]["kernel_us_per_step"],
      d["policy_rollout"]["kernel_us_per_step"]))
PY
  done
done
