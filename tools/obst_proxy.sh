#!/bin/bash
# Step-kernel time against per-lane obstacle work: the same kernel built for 13+5 and for 7+3
# obstacles (tools/build_variants.sh o135 / o73), plus phase-skip masks on the 13+5 diagnostics
# build (o135s); tools/ablate.py, graph-replayed, 65 536 envs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/obst
run() {  # name lib obst masks
  BALLENV_LIB=tools/diag/$2/libballenv.so OBST=$3 MASKS=$4 SIZES=65536 GRAPH=1 timeout -k 10 120 python3 tools/ablate.py \
      > gpurun_out/obst/$1.txt 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "$1 rc=$rc"; tail -5 gpurun_out/obst/$1.txt; exit $rc; }
  grep envs gpurun_out/obst/$1.txt | sed "s/^/[$1] /"
}
run o135 o135 13,5 0
run o73 o73 7,3 0
run o135s o135s 13,5 0,1,2,4,8,16,32,6,14
