#!/bin/bash
# Round-3 counters of the config-5 fused policy rollout and the createBoard kernels (after the
# VGPR-form change), plus the fused rollouts' phase stamps (stamps build tools/diag/st).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3q; mkdir -p $O; export TMPDIR=/tmp
BALLENV_LIB=tools/diag/st/libballenv.so timeout -k 10 300 python tools/fused_phases.py > $O/fused_phases.txt 2>&1
rc=$?; echo "phases rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/fused_phases.txt; exit $rc; }
timeout -k 10 900 bash tools/pmc_passes.sh r3q/pmc --no-cpu-baseline --steps 10 --warmup 2 --settle 10 \
    --policy-steps 200 --torch-policy-steps 0 --board-steps 200 --rollout-steps 0 --cold-steps 0 \
    --config2-steps 0 --large-steps 0 --from-reset-steps 0 --blocks-launches 0
rc=$?; echo "pmc rc=$rc"; [ $rc -ne 0 ] && exit $rc
python tools/pmc_report.py $O/pmc "rollout_kernel<10, 13, 5, 13, 2, 10>" 6553600 --first 4 --out $O/r03_pmc_policy_rollout.json > /dev/null
python tools/pmc_report.py $O/pmc "board_kernel<6, false" 65536 --out $O/r03_pmc_board_step.json > /dev/null
python tools/pmc_report.py $O/pmc "board_kernel<6, true" 6553600 --out $O/r03_pmc_board_rollout.json > /dev/null
ls $O
