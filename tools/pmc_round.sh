#!/bin/bash
# A round's HBM counters (ROUND=r06) of every step-API and fused kernel whose name or size is new this
# round, from ONE pair of FETCH_SIZE / WRITE_SIZE passes (tools/pmc_passes.sh) on one bench.py command:
#   headline step2_kernel<..., true> at 65 536 envs        -> ROUND_pmc_step_kernel.json
#     (the same kernel and size is config 4's 4-GPU shard   -> ROUND_pmc_config4_65536.json)
#   config 4's 8-GPU shard, 32 768 envs                     -> ROUND_pmc_config4_32768.json
#   config 2, stepw_kernel<5, 13, 5, 8, true>, 4 096 envs   -> ROUND_pmc_config2.json
#   fused rollout at config 2 (rolloutw_kernel, 4 096 envs) -> ROUND_pmc_rollout_config2.json
#   fused rollout at the 32 768-env shard                   -> ROUND_pmc_rollout_shard_32768.json
#   the autoreset pool's fill at 65 536 envs                -> ROUND_pmc_pool_fill.json
# bench.py reads them back through newest_pmc() (kernel name + units per dispatch must match).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=${ROUND:-r06}; O=gpurun_out/${R}_pmcr; mkdir -p $O
PASSES="FETCH_SIZE WRITE_SIZE" timeout -k 10 500 bash tools/pmc_passes.sh ${R}_pmcr/p --no-cpu-baseline --steps 200 \
    --warmup 20 --settle 10 --policy-steps 0 --torch-policy-steps 0 --board-steps 0 --rollout-steps 200 --rollout-chunk 100 \
    --cold-steps 0 --config2-steps 200 --config4-steps 200 --config4-envs 32768 --large-steps 0 --from-reset-steps 0 \
    --blocks-launches 0 --shard-steps 0 --eager-steps 0 || exit 1
rep() { python3 tools/pmc_report.py $O/p "$1" $2 --grid $3 --out $O/${R}_pmc_$4.json | tail -3; }
rep "step2_kernel<10, 13, 5, true>" 65536 131072 step_kernel
cp $O/${R}_pmc_step_kernel.json $O/${R}_pmc_config4_65536.json
rep "step2_kernel<10, 13, 5, true>" 32768 65536 config4_32768
rep "stepw_kernel<5, 13, 5, 8, true>" 4096 32768 config2
rep "rolloutw_kernel<5, 13, 5, 8>" 409600 32768 rollout_config2
rep "rollout_kernel<10, 13, 5, 0, 1, 10>" 3276800 32768 rollout_shard_32768
rep "pool_fill_kernel<10, 13, 5>" 65536 65536 pool_fill
