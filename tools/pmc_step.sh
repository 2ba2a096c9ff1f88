#!/bin/bash
# PMC passes over tools/microbench (each pass its own rocprofv3 run; --pmc with kernel trace only).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc; export TMPDIR=/tmp
rocprofv3 -L > gpurun_out/pmc/counters_list.txt 2>&1 || true
i=0
for set in "${@}"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmc/p$i -o run -- ./tools/microbench > gpurun_out/pmc/p$i.log 2>&1
  rc=$?; echo "pass $i ($set) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmc/p$i.log; exit $rc; fi
done
