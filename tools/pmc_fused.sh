#!/bin/bash
# A round's PMC of the two fused rollouts (ROUND=r04): the random-action be_rollout kernel and the
# config-5 be_policy_rollout kernel at 65 536 envs, W=10, 100-step launches -- HBM bytes and the SQ
# instruction / cycle counters (tools/pmc_passes.sh, one rocprofv3 run per pass) -> per-kernel JSON.
# The policy report takes the leg's first 6 dispatches: the 7th is a recorded-obs launch (+104 B/env-step of obs).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=${ROUND:-r04}; O=gpurun_out/${R}_pmc; mkdir -p $O; export TMPDIR=/tmp
PASSES="FETCH_SIZE WRITE_SIZE sq1 sq2" timeout -k 10 900 bash tools/pmc_passes.sh ${R}_pmc/fused --no-cpu-baseline --steps 10 \
    --warmup 2 --settle 10 --policy-steps 300 --torch-policy-steps 0 --board-steps 0 --rollout-steps 300 --cold-steps 0 \
    --config2-steps 0 --config4-steps 0 --large-steps 0 --from-reset-steps 0 --blocks-launches 0 || exit 1
python3 tools/pmc_report.py $O/fused "rollout_kernel<10, 13, 5, 0," 6553600 --out $O/${R}_pmc_rollout_kernel.json | tail -2
python3 tools/pmc_report.py $O/fused "rollout_kernel<10, 13, 5, 13," 6553600 --first 6 --out $O/${R}_pmc_policy_rollout.json | tail -2
