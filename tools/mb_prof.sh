#!/bin/bash
# microbench under rocprofv3 kernel trace, one run per debug mask
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/mbprof; export TMPDIR=/tmp
for m in "$@"; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/mbprof/m$m -o run -- ./tools/${MB:-microbench} $m > gpurun_out/mbprof/m$m.log 2>&1
  rc=$?; echo "mask $m rc=$rc"; grep envs gpurun_out/mbprof/m$m.log
  [ $rc -ne 0 ] && exit $rc
  python3 - "$m" <<'PY'
import csv, sys, statistics, collections
m = sys.argv[1]
rows = list(csv.DictReader(open(f"gpurun_out/mbprof/m{m}/run_kernel_trace.csv")))
d = collections.defaultdict(list)
for r in rows:
    d[(r["Kernel_Name"][:40], r["Grid_Size_X"] if "Grid_Size_X" in r else r.get("Grid_Size", ""))].append(
        (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0)
for k, v in sorted(d.items()):
    if len(v) > 10:
        print(f"  {k[0]:40s} grid={k[1]:>8s} n={len(v):4d} median_us={statistics.median(v):8.2f}")
PY
done
