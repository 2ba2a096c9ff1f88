#!/bin/bash
# Four-lanes-per-env proxy (tools/build_variants.sh s4 / s4d): parity against step2_kernel,
# then graph-replayed launch times (tools/ablate.py) for 1 / 2 / 4 lanes per env.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s4
BALLENV_LIB=tools/diag/s4/libballenv.so timeout -k 10 120 python3 tools/step4_check.py > gpurun_out/s4/check.txt 2>&1
rc=$?; tail -2 gpurun_out/s4/check.txt; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  BALLENV_LIB=tools/diag/s4/libballenv.so LPES=1,2,4 MASKS=0 SIZES=65536,98304,131072 GRAPH=1 timeout -k 10 120 \
      python3 tools/ablate.py > gpurun_out/s4/time$r.txt 2>&1 || exit $?
  cat gpurun_out/s4/time$r.txt | grep envs
done
BALLENV_LIB=tools/diag/s4d/libballenv.so LPES=2,4 MASKS=0,1 SIZES=65536 GRAPH=1 timeout -k 10 120 \
    python3 tools/ablate.py > gpurun_out/s4/diag.txt 2>&1 || exit $?
grep envs gpurun_out/s4/diag.txt
