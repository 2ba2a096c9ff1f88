#!/bin/bash
# Step-kernel time against the obs copy's cache-policy bits (tools/build_variants.sh auxN builds,
# o135 = the default 16 = sc1) and without the copy (o135s, DBG_NO_COPY); tools/ablate.py, graph-replayed.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/aux
for r in 1 2; do
for v in ${VARIANTS:-o135 aux0 aux1 aux2 aux17 aux18}; do
  BALLENV_LIB=tools/diag/$v/libballenv.so MASKS=0 SIZES=65536,262144 GRAPH=1 timeout -k 10 120 python3 tools/ablate.py \
      > gpurun_out/aux/$v.txt 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "$v rc=$rc"; tail -5 gpurun_out/aux/$v.txt; exit $rc; }
  grep envs gpurun_out/aux/$v.txt | sed "s/^/[$v r$r] /"
done
done
BALLENV_LIB=tools/diag/o135s/libballenv.so MASKS=0,32768,1,32769 SIZES=65536 GRAPH=1 timeout -k 10 120 python3 tools/ablate.py \
    > gpurun_out/aux/nocopy.txt 2>&1 || exit $?
grep envs gpurun_out/aux/nocopy.txt | sed "s/^/[o135s] /"
