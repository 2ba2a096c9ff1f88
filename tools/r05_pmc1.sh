#!/bin/bash
# Round-5 PMC refresh, part 1: the headline step kernel (tools/pmc_bench.sh) and config 4's per-rank
# shard sizes (tools/pmc_config4.sh, ROUND=r05), FETCH_SIZE / WRITE_SIZE passes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
timeout -k 10 500 bash tools/pmc_bench.sh || exit 1
ROUND=r05 SIZES="${SIZES:-32768 65536 131072 262144}" timeout -k 10 700 bash tools/pmc_config4.sh || exit 1
