#!/bin/bash
# Round-5 PMC refresh, part 2: config 2 (stepw_kernel) and the 2^20-env large batch (one-lane kernel),
# and the createBoard step / fused kernels -- tools/round_pmc.sh's passes without the headline one.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=r05; O=gpurun_out/${R}_pmc; mkdir -p $O; export TMPDIR=/tmp
PASSES="FETCH_SIZE WRITE_SIZE" timeout -k 10 600 bash tools/pmc_passes.sh ${R}_pmc/c2 --no-cpu-baseline --steps 10 --warmup 2 --settle 10 \
    --policy-steps 0 --torch-policy-steps 0 --board-steps 0 --rollout-steps 0 --cold-steps 0 --config4-steps 0 --from-reset-steps 0 \
    --blocks-launches 0 --shard-steps 0 --eager-steps 0 --config2-steps 200 --large-steps 100 || exit 1
python3 tools/pmc_report.py $O/c2 "stepw_kernel<5, 13, 5, 8>" 4096 --out $O/${R}_pmc_config2.json | tail -2
python3 tools/pmc_report.py $O/c2 "be_kernel<10, 0, 13, 5>" 1048576 --out $O/${R}_pmc_large_batch.json | tail -2
PASSES="FETCH_SIZE WRITE_SIZE sq1 sq2" timeout -k 10 900 bash tools/pmc_passes.sh ${R}_pmc/board --no-cpu-baseline --steps 10 --warmup 2 \
    --settle 10 --policy-steps 0 --torch-policy-steps 0 --board-steps 200 --board-cpu-seconds 0 --rollout-steps 0 --cold-steps 0 \
    --config2-steps 0 --config4-steps 0 --large-steps 0 --from-reset-steps 0 --blocks-launches 0 --shard-steps 0 --eager-steps 0 || exit 1
python3 tools/pmc_report.py $O/board "board_kernel<6, false" 65536 --out $O/${R}_pmc_board_step.json | tail -2
python3 tools/pmc_report.py $O/board "board_kernel<6, true" 6553600 --out $O/${R}_pmc_board_rollout.json | tail -2
