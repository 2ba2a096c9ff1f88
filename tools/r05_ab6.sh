#!/bin/bash
# Round-5 step2 span-table raster: the step2 / parity GPU tests, then a 3x interleaved A/B of the
# headline, config-2 and config-4 shard legs against tools/diag/base (HEAD before the change).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05_f}; mkdir -p $O
timeout -k 10 500 python -u -m pytest ${TESTS:-tests/test_gpu_episode.py tests/test_gpu_parity.py} -m gpu -x -q -p no:cacheprovider --timeout 150 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
B="${B:-base}" REPS=${REPS:-3} bash tools/legs_ab.sh
