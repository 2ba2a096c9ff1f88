#!/bin/bash
# step2_kernel phase ablation at the config-4 shard (32 768) and headline (65 536) sizes on the skip
# library (-DBE_DIAG_SKIP; outputs wrong whenever a bit is set), graph-replayed launches, median of 5.
# masks: 0 full, 8 no Philox, 2 no raster, 4 no obs (return before it), 32768 no copy-out, 1 no stats,
# 16384 no reset, 256 exit after the physics, 128 exit after the table barrier, 64 exit at entry.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05_ablate; mkdir -p $O
BALLENV_LIB=tools/diag/skip/libballenv.so GRAPH=1 MASKS=0,8,2,4,32768,1,16384,256,128,64 SIZES=32768,65536 W=10 \
  timeout -k 10 300 python3 tools/ablate.py > $O/step2.txt 2>&1 || { tail -5 $O/step2.txt; exit 1; }
cat $O/step2.txt
