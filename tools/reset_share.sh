#!/bin/bash
# How much of each step kernel's time the autoreset pass costs: the skip-diagnostics library
# (tools/diag/skip, -DBE_DIAG_SKIP) with and without DBG_NO_RESET (16384), graph-replayed launches,
# at the headline (65536 W=10), config-4 shard (32768 W=10) and config-2 (4096 W=5) sizes; then the
# createBoard step with and without autoreset (release library).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/reset_share; mkdir -p $O
BALLENV_LIB=tools/diag/skip/libballenv.so GRAPH=1 MASKS=0,16384 SIZES=65536,32768 W=10 timeout -k 10 200 python3 tools/ablate.py > $O/w10.txt 2>&1 || { tail -5 $O/w10.txt; exit 1; }
grep envs $O/w10.txt
BALLENV_LIB=tools/diag/skip/libballenv.so GRAPH=1 MASKS=0,16384 SIZES=4096 W=5 timeout -k 10 200 python3 tools/ablate.py > $O/w5.txt 2>&1 || { tail -5 $O/w5.txt; exit 1; }
grep envs $O/w5.txt
timeout -k 10 200 python3 tools/board_ablate.py > $O/board.txt 2>&1 || { tail -5 $O/board.txt; exit 1; }
grep features $O/board.txt
