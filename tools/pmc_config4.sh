#!/bin/bash
# HBM traffic of BASELINE config 4's step kernels at each per-rank shard of the fixed 262 144-env
# batch: 262 144 (N = 1), 131 072 (N = 2), 65 536 (N = 4) and 32 768 (N = 8) envs on one GPU, from
# FETCH_SIZE / WRITE_SIZE passes on bench.py's config4 leg (tools/pmc_passes.sh, pmc_report.py);
# out: gpurun_out/pmc_c4/ROUND_pmc_config4_<envs>.json (bench.py's config4 leg reads
# profiles/ROUND_pmc_config4_<envs per rank>.json).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=${ROUND:-r04}
COMMON="--no-cpu-baseline --steps 10 --warmup 2 --settle 10 --policy-steps 0 --torch-policy-steps 0 --board-steps 0 --rollout-steps 0 --cold-steps 0 --config2-steps 0 --large-steps 0 --from-reset-steps 0 --blocks-launches 0 --shard-steps 0 --eager-steps 0 --config4-steps 200"
for n in ${SIZES:-262144 131072 65536 32768}; do
  PASSES="FETCH_SIZE WRITE_SIZE" timeout -k 10 400 bash tools/pmc_passes.sh pmc_c4/g$n $COMMON --config4-envs $n || exit 1
  # grid = the kernel's threads at this size (step2: 2 lanes per env, 128-env blocks; one lane: 256-env blocks)
  k="be_kernel<10, 0, 13, 5, $([ $n -le 131072 ] && echo true || echo false)>"; g=$(( (n + 255) / 256 * 256 ))
  [ $n -le 98304 ] && { k="step2_kernel<10, 13, 5, true>"; g=$(( (n + 127) / 128 * 256 )); }
  python3 tools/pmc_report.py gpurun_out/pmc_c4/g$n "$k" $n --grid $g --out gpurun_out/pmc_c4/${R}_pmc_config4_$n.json | tail -2
done
