#!/bin/bash
# createBoard after the single-chain resets: phase stamps with resets per wave, and the counters
# of both board kernels (refreshes r03_pmc_board_step / r03_pmc_board_rollout).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3v; mkdir -p $O; export TMPDIR=/tmp
BALLENV_LIB=tools/diag/st/libballenv.so timeout -k 10 200 python tools/board_phases.py > $O/board_phases.txt 2>&1
rc=$?; grep -v amdgpu.ids $O/board_phases.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 bash tools/pmc_passes.sh r3v/pmc --no-cpu-baseline --steps 10 --warmup 2 --settle 10 \
    --policy-steps 0 --torch-policy-steps 0 --board-steps 200 --rollout-steps 0 --cold-steps 0 \
    --config2-steps 0 --large-steps 0 --from-reset-steps 0 --blocks-launches 0
rc=$?; echo "pmc rc=$rc"; [ $rc -ne 0 ] && exit $rc
python tools/pmc_report.py $O/pmc "board_kernel<6, false" 65536 --out $O/r03_pmc_board_step.json > /dev/null
python tools/pmc_report.py $O/pmc "board_kernel<6, true" 6553600 --out $O/r03_pmc_board_rollout.json > /dev/null
ls $O
