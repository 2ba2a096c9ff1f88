#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel trace of the bench.
# Every GPU step has its own time limit; a crash/timeout stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc"
  if [ $rc -gt 1 ]; then echo "stopping after $name (rc=$rc)"; tail -20 "gpurun_out/$name.log"; exit $rc; fi
  return 0
}
TAG=${TAG:-run}
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  step pytest_gpu 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 120 --timeout-method thread ${PYTEST_ARGS:-}
  tail -3 gpurun_out/pytest_gpu.log
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
step bench_driver 300 python bench.py --gpus 1 --steps 20 --warmup 5 ${BENCH_ARGS:-}
tail -1 gpurun_out/bench_driver.log
step bench 400 python bench.py ${BENCH_ARGS:-}
tail -1 gpurun_out/bench.log
if [ "${PROFILE:-1}" = "1" ]; then
  # headline step kernel alone (no other leg), then the config-5 policy rollouts (two-launch and
  # fused) with the fused random-action rollout
  step rocprof 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- \
      python bench.py --no-cpu-baseline --steps 300 --warmup 20 --policy-steps 0 --board-steps 0 --rollout-steps 0 ${BENCH_ARGS:-}
  find gpurun_out/prof_$TAG -name "*kernel_stats.csv" -exec head -4 {} \;
  step rocprof_policy 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG}_policy -o run -- \
      python bench.py --no-cpu-baseline --steps 10 --warmup 5 --policy-steps 200 --torch-policy-steps 0 --board-steps 0 \
      --rollout-steps 1000 ${BENCH_ARGS:-}
  find gpurun_out/prof_${TAG}_policy -name "*kernel_stats.csv" -exec head -4 {} \;
fi
if [ "${PMC:-1}" = "1" ]; then
  step pmc 700 bash tools/pmc_bench.sh
  tail -1 gpurun_out/pmc.log
fi
