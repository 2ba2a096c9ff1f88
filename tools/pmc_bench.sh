#!/bin/bash
# HBM-side traffic of the step kernel, measured on bench.py itself (eager launches):
# one rocprofv3 pass per counter (FETCH_SIZE and WRITE_SIZE don't fit one pass), kernel
# trace only -- then tools/pmc_summary.py -> gpurun_out/pmc/pmc_step_kernel.json
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc; export TMPDIR=/tmp
ARGS="--no-cpu-baseline --mode eager --steps 200 --warmup 20 --policy-steps 0 --board-steps 0 --rollout-steps 0 --cold-steps 0 --config2-steps 0 --config4-steps 0 --large-steps 0 --from-reset-steps 0 --blocks-launches 0 --shard-steps 0 --eager-steps 0 ${BENCH_ARGS:-}"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc/$c -o run -- python3 bench.py $ARGS \
      > gpurun_out/pmc/$c.log 2>&1
  rc=$?; echo "pass $c rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmc/$c.log; exit $rc; fi
done
python3 tools/pmc_summary.py gpurun_out/pmc $ARGS
