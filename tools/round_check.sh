#!/bin/bash
# A round GPU session (ROUND=r04 names the output dir): GPU tests, smoke, the driver-shaped and default bench lines, rocprofv3 kernel
# stats (headline; config 2 + large batch; fused legs), PMC passes (config 2 / large batch / the
# headline step kernel).  Every GPU step under its own time limit; a crash/timeout stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/${ROUND:-r04}_check
export TMPDIR=/tmp
O=gpurun_out/${ROUND:-r04}_check
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc"
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; tail -20 "$O/$name.log"; exit $rc; fi
  return 0
}
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  step pytest_gpu 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 120 --timeout-method thread
  tail -2 $O/pytest_gpu.log
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
step bench_driver 300 python bench.py --gpus 1 --steps 20 --warmup 5
tail -c 400 $O/bench_driver.log; echo
step bench 400 python bench.py
tail -c 400 $O/bench.log; echo
if [ "${PROFILE:-1}" = "1" ]; then
  step rocprof 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_head -o run -- \
      python bench.py --no-cpu-baseline --steps 300 --warmup 20 --policy-steps 0 --board-steps 0 --rollout-steps 0 \
      --cold-steps 0 --config2-steps 1000 --large-steps 200 --from-reset-steps 0 --blocks-launches 0
  find $O/prof_head -name "*kernel_stats.csv" -exec head -6 {} \;
  step rocprof_fused 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_fused -o run -- \
      python bench.py --no-cpu-baseline --steps 10 --warmup 5 --policy-steps 200 --torch-policy-steps 0 --board-steps 200 \
      --rollout-steps 1000 --cold-steps 0 --config2-steps 0 --large-steps 0 --from-reset-steps 0 --blocks-launches 0
  find $O/prof_fused -name "*kernel_stats.csv" -exec head -8 {} \;
fi
if [ "${PMC:-1}" = "1" ]; then
  step pmc_c2_large 600 bash tools/pmc_passes.sh ${ROUND:-r04}_check/pmc --no-cpu-baseline --steps 10 --warmup 2 --settle 10 --policy-steps 0 \
      --board-steps 0 --rollout-steps 0 --cold-steps 0 --from-reset-steps 0 --blocks-launches 0 --config2-steps 200 --large-steps 100
  python tools/pmc_report.py $O/pmc "stepw_kernel<5, 13, 5, 8>" 4096 --out $O/${ROUND:-r04}_pmc_config2.json > /dev/null
  python tools/pmc_report.py $O/pmc "be_kernel<10, 0, 13, 5, true>" 1048576 --out $O/${ROUND:-r04}_pmc_large_batch.json > /dev/null
  step pmc_step 700 bash tools/pmc_bench.sh
  tail -1 $O/pmc_step.log
fi
