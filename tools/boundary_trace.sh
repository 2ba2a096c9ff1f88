#!/bin/bash
# What happens at a graph boundary: kernel + memory-copy + HIP API trace of back-to-back
# 20-launch graph replays (tools/short_graph.py span).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/btrace; export TMPDIR=/tmp
K=20 KINDS=span timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace --output-format csv \
    -d gpurun_out/btrace/run -o run -- python3 tools/short_graph.py > gpurun_out/btrace/log.txt 2>&1 || exit $?
ls -R gpurun_out/btrace | head -20
