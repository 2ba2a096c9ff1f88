#!/bin/bash
# rocprofv3 kernel-trace medians for each tools/mb_* variant binary given as args
# (an arg "bin@VAR=value" runs tools/bin with that environment variable set)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/mbv; export TMPDIR=/tmp
for spec in "$@"; do
  bin=${spec%%@*}; b=${spec//[@=]/_}
  if [ "$bin" != "$spec" ]; then export "${spec#*@}"; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/mbv/$b -o run -- ./tools/$bin 0 > gpurun_out/mbv/$b.log 2>&1
  if [ "$bin" != "$spec" ]; then v=${spec#*@}; unset "${v%%=*}"; fi
  rc=$?; echo "== $b rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/mbv/$b.log; exit $rc; }
  python3 - "$b" <<'PY'
import csv, sys, statistics, collections
b = sys.argv[1]
d = collections.defaultdict(list)
for r in csv.DictReader(open(f"gpurun_out/mbv/{b}/run_kernel_trace.csv")):
    d[(r["Kernel_Name"][:45], r.get("Grid_Size_X") or r.get("Grid_Size", ""))].append(
        (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0)
for k, v in sorted(d.items()):
    if len(v) > 10 :
        print(f"  {k[0]:34s} grid={k[1]:>8s} n={len(v):4d} median_us={statistics.median(v):8.2f} p90={sorted(v)[int(.9*len(v))]:8.2f}")
PY
done
