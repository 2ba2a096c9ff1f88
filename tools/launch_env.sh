#!/bin/bash
# HIP runtime launch settings vs the step API's fixed costs: for each setting, the short-region
# costs (tools/sync_cost.py) and the bench's driver-shaped (20-step) and 1000-step lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/launch_env
for spec in ${SPECS:-default: batch1:DEBUG_HIP_GRAPH_BATCH_SIZE=1 batch4:DEBUG_HIP_GRAPH_BATCH_SIZE=4 devkernarg:HIP_FORCE_DEV_KERNARG=1 hostkernarg:HIP_FORCE_DEV_KERNARG=0 nocapture:DEBUG_CLR_GRAPH_PACKET_CAPTURE=0}; do
  name=${spec%%:*}; vars=${spec#*:}   # name:VAR=value (one variable)
  o=gpurun_out/launch_env/$name
  env $vars timeout -k 10 120 python3 tools/sync_cost.py > $o.sync.txt 2>&1
  rc=$?; echo "[$name] sync_cost rc=$rc"; [ $rc -ne 0 ] && { tail -5 $o.sync.txt; exit $rc; }
  env $vars timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 20 --warmup 5 --policy-steps 0 --board-steps 0 \
      --rollout-steps 0 > $o.b20.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "[$name] b20 rc=$rc"; tail -5 $o.b20.log; exit $rc; }
  env $vars timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 1000 --warmup 100 --policy-steps 0 \
      --board-steps 0 --rollout-steps 1000 > $o.b1000.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "[$name] b1000 rc=$rc"; tail -5 $o.b1000.log; exit $rc; }
  python3 - "$name" "$o" <<'EOF'
import json, sys
name, o = sys.argv[1], sys.argv[2]
for k in ("b20", "b1000"):
    d = json.loads(open(f"{o}.{k}.log").read().strip().splitlines()[-1])
    f = d.get("fused_rollout") or {}
    print(f"[{name}] {k}: {d['value']:.3e} env-steps/s, {d['ms_per_step'] * 1e3:.2f} us/step wall, kernel "
          f"{d['roofline']['kernel_us_mean']:.2f} us" + (f", fused {f['kernel_us_per_step']:.2f} us" if f else ""))
EOF
  grep -E "host time|raw|graph end=sync" $o.sync.txt | sed "s/^/[$name] /"
done
