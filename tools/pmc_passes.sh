#!/bin/bash
# rocprofv3 --pmc passes (one run per pass, kernel trace only) on one bench.py command:
#   usage: tools/pmc_passes.sh <out dir under gpurun_out> <bench.py args...>
# pass sq1/sq2: SQ instruction, cycle, MFMA and LDS counters (+ GRBM clock); FETCH_SIZE, WRITE_SIZE:
# HBM-side bytes.  tools/pmc_report.py turns the passes into a per-kernel JSON.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"; export TMPDIR=/tmp
declare -A P
P[sq1]="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY"
P[sq2]="SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT"
P[FETCH_SIZE]="FETCH_SIZE"
P[WRITE_SIZE]="WRITE_SIZE"
for name in ${PASSES:-sq1 sq2 FETCH_SIZE WRITE_SIZE}; do
  timeout -s KILL 180 rocprofv3 --pmc ${P[$name]} --output-format csv -d "$OUT/$name" -o run -- python3 bench.py "$@" \
      > "$OUT/$name.log" 2>&1
  rc=$?; echo "pass $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/$name.log"; exit $rc; fi
done
exit 0
