#!/bin/bash
# SQ instruction / cycle counters of the step kernel, one rocprofv3 --pmc pass per kernel variant
# (8 SQ counters = one pass): eager bench.py launches, kernel trace only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmcsq; export TMPDIR=/tmp
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU"
ARGS="--no-cpu-baseline --mode eager --steps 200 --warmup 20 --policy-steps 0 --board-steps 0 --rollout-steps 0"
for L in ${LPES:-1 2}; do
  BALLENV_STEP_LPE=$L timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmcsq/lpe$L -o run -- \
      python3 bench.py $ARGS > gpurun_out/pmcsq/lpe$L.log 2>&1
  rc=$?; echo "pmc LPE=$L rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/pmcsq/lpe$L.log; exit $rc; }
done
exit 0
