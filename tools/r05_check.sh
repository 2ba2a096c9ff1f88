#!/bin/bash
# Round-5 GPU session: the new GPU tests first, then the whole GPU suite, the default bench line, and
# per-wave phase stamps of step2_kernel at the config-4 shard size (32 768 envs) and the headline
# size (65 536) from the -DBE_DIAG_STAMPS library (BUILD=1 bash tools/stamps_run.sh here first).
# SKIP_SUITE=1 skips the whole-suite step; STAMPS_ONLY=1 runs only the stamps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-r05_a}; mkdir -p $O; export TMPDIR=/tmp
if [ "${STAMPS_ONLY:-0}" != "1" ]; then
  timeout -k 10 400 python -u -m pytest ${NEW_TESTS:-tests/test_gpu_coord_range.py tests/test_bench_contract.py} -m gpu -x -v \
      -p no:cacheprovider --timeout 150 --timeout-method thread > $O/pytest_new.log 2>&1
  rc=$?; tail -3 $O/pytest_new.log; [ $rc -ne 0 ] && { grep -E "^E |FAIL|Error" $O/pytest_new.log | head -30; exit $rc; }
  if [ "${SKIP_SUITE:-0}" != "1" ]; then
    timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 150 --timeout-method thread \
        > $O/pytest_gpu.log 2>&1
    rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -ne 0 ] && { grep -E "^E |FAIL" $O/pytest_gpu.log | head -30; exit $rc; }
  fi
  timeout -k 10 400 python bench.py > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
  tail -c 300 $O/bench.log; echo
fi
for n in ${STAMP_SIZES:-32768 65536}; do
  BALLENV_STEP_LPE=2 timeout -k 10 120 ./tools/stamps $n > $O/stamps_step2_$n.txt 2>&1
  rc=$?; echo "stamps $n rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/stamps_step2_$n.txt; exit $rc; }
done
exit 0
