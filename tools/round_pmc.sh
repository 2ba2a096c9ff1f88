#!/bin/bash
# A round's PMC refresh (ROUND=r04): HBM bytes (FETCH_SIZE / WRITE_SIZE passes) of the headline step
# kernel (tools/pmc_bench.sh -> gpurun_out/pmc/pmc_step_kernel.json), config 2 + the 2^20-env point and
# the createBoard step / fused kernels (tools/pmc_passes.sh + pmc_report.py), each GPU step under its own
# time limit; bench.py reads the copies committed under profiles/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=${ROUND:-r04}; O=gpurun_out/${R}_pmc; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 700 bash tools/pmc_bench.sh || exit 1
tail -1 gpurun_out/pmc/FETCH_SIZE.log > /dev/null
PASSES="FETCH_SIZE WRITE_SIZE" timeout -k 10 600 bash tools/pmc_passes.sh ${R}_pmc/c2 --no-cpu-baseline --steps 10 --warmup 2 --settle 10 \
    --policy-steps 0 --torch-policy-steps 0 --board-steps 0 --rollout-steps 0 --cold-steps 0 --config4-steps 0 --from-reset-steps 0 \
    --blocks-launches 0 --shard-steps 0 --eager-steps 0 --config2-steps 200 --large-steps 100 || exit 1
python3 tools/pmc_report.py $O/c2 "stepw_kernel<5, 13, 5, 8>" 4096 --out $O/${R}_pmc_config2.json | tail -2
python3 tools/pmc_report.py $O/c2 "be_kernel<10, 0, 13, 5, true>" 1048576 --out $O/${R}_pmc_large_batch.json | tail -2
PASSES="FETCH_SIZE WRITE_SIZE sq1 sq2" timeout -k 10 900 bash tools/pmc_passes.sh ${R}_pmc/board --no-cpu-baseline --steps 10 --warmup 2 \
    --settle 10 --policy-steps 0 --torch-policy-steps 0 --board-steps 200 --board-cpu-seconds 0 --rollout-steps 0 --cold-steps 0 \
    --config2-steps 0 --config4-steps 0 --large-steps 0 --from-reset-steps 0 --blocks-launches 0 --shard-steps 0 --eager-steps 0 || exit 1
python3 tools/pmc_report.py $O/board "board_kernel<6, false, 1, true>" 65536 --out $O/${R}_pmc_board_step.json | tail -2
python3 tools/pmc_report.py $O/board "board_kernel<6, true" 6553600 --out $O/${R}_pmc_board_rollout.json | tail -2
