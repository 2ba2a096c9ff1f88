#!/bin/bash
# SQ counter passes (sq1, sq2) of step2_kernel on the config-4 leg at ENVS4 envs (default 32 768):
# instructions per wave and the wave-cycle split (active / waiting) -- tools/pmc_report.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
n=${ENVS4:-32768}; O=r05_sq/g$n
PASSES="sq1 sq2" timeout -k 10 400 bash tools/pmc_passes.sh $O --no-cpu-baseline --steps 10 --warmup 2 --settle 10 --policy-steps 0 \
  --torch-policy-steps 0 --board-steps 0 --rollout-steps 0 --cold-steps 0 --config2-steps 0 --large-steps 0 --from-reset-steps 0 \
  --blocks-launches 0 --shard-steps 0 --eager-steps 0 --config4-steps 200 --config4-envs $n || exit 1
python3 tools/pmc_report.py gpurun_out/$O "step2_kernel<10, 13, 5>" $n --out gpurun_out/$O/sq_step2_$n.json
