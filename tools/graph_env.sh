#!/bin/bash
# HIP runtime settings vs the GPU-side cost of a graph boundary: tools/short_graph.py (span, b2b)
# at 20 and 100 launches per graph, one process per setting.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/genv
for spec in ${SPECS:-default: fgq1:DEBUG_HIP_FORCE_GRAPH_QUEUES=1 hdp0:DEBUG_CLR_KERNARG_HDP_FLUSH_WA=0 hdp1:DEBUG_CLR_KERNARG_HDP_FLUSH_WA=1 kcopy0:DEBUG_HIP_KERNARG_COPY_OPT=0 kcopy1:DEBUG_HIP_KERNARG_COPY_OPT=1 batch64:DEBUG_HIP_GRAPH_BATCH_SIZE=64}; do
  name=${spec%%:*}; vars=${spec#*:}
  for K in 20 100; do
    env $vars K=$K KINDS="span b2b" timeout -k 10 100 python3 tools/short_graph.py > gpurun_out/genv/$name.k$K.txt 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "[$name] K=$K rc=$rc"; tail -5 gpurun_out/genv/$name.k$K.txt; exit $rc; }
    grep us/step gpurun_out/genv/$name.k$K.txt | sed "s/^/[$name K=$K] /"
  done
done
