#!/bin/bash
# Round-5 one-lane fixed kernel span-table raster: GPU tests, then a 3x interleaved A/B of config 4
# on one rank at 131 072 envs and the 2^20-env large batch against tools/diag/base.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05_g}; mkdir -p $O
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_episode.py tests/test_gpu_parity.py tests/test_gpu_coord_range.py} -m gpu -x -q -p no:cacheprovider --timeout 150 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
B="${B:-base}" REPS=${REPS:-3} ENVS4=${ENVS4:-131072} bash tools/big_ab.sh
