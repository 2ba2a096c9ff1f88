#!/bin/bash
# One box session: A/B of variant libraries on the headline leg (tools/ab_bench.sh), the episode parity
# tests on the first variant (PARITY_LIB), then the whole-round refresh (tools/gpu_check.sh).
# Any GPU step that fails with a crash / abort / timeout ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/ab_bench.sh "$@" > gpurun_out/ab_variants.txt 2>&1
rc=$?; cat gpurun_out/ab_variants.txt; [ $rc -ne 0 ] && { echo "ab rc=$rc"; exit $rc; }
for lib in ${PARITY_LIB:-}; do   # space-separated variant libraries
  n=$(basename "$(dirname "$lib")")
  BALLENV_LIB=$lib timeout -k 10 400 python -u -m pytest tests/test_gpu_episode.py -x -q -p no:cacheprovider \
      --timeout 120 --timeout-method thread > gpurun_out/variant_parity_$n.log 2>&1
  rc=$?; echo "parity $n rc=$rc"; tail -2 gpurun_out/variant_parity_$n.log; [ $rc -gt 1 ] && exit $rc
done
[ "${CHECK:-1}" = "1" ] || exit 0
TAG=${TAG:-run} bash tools/gpu_check.sh
