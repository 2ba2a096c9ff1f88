#!/bin/bash
# Where config 2's read traffic comes from: FETCH_SIZE / WRITE_SIZE of stepw_kernel<5, 13, 5, 8>
# (4 096 envs, graph-replayed launches through tools/ablate.py) on the skip-diagnostics library
# (tools/diag/skip, -DBE_DIAG_SKIP), one process per phase-skip mask:
#   0 full step | 256 return after the physics, stores and stats | 4 no obs | 16384 no reset pass
#   1 no stats fold | 128 return right after the loads (consumes some of them)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/pmc_stepw; mkdir -p $O; export TMPDIR=/tmp
for m in ${MASKS:-0 256 4 16384 1 128}; do
  for c in FETCH_SIZE WRITE_SIZE; do
    BALLENV_LIB=tools/diag/skip/libballenv.so GRAPH=1 MASKS=$m SIZES=4096 W=5 timeout -s KILL 120 \
        rocprofv3 --pmc $c --output-format csv -d $O/m${m}_$c -o run -- python3 tools/ablate.py > $O/m${m}_$c.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "mask $m $c rc=$rc"; tail -5 $O/m${m}_$c.log; exit $rc; }
  done
done
python3 - $O <<'PY'
import csv, glob, statistics, sys, collections
O = sys.argv[1]
rows = {}
for d in sorted(glob.glob(f"{O}/m*_*/")):
    m, c = d.rstrip("/").split("/")[-1][1:].split("_", 1)
    per = collections.defaultdict(float)
    for f in glob.glob(d + "**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "stepw_kernel" in r["Kernel_Name"]:
                per[int(r["Dispatch_Id"])] += float(r["Counter_Value"])
    v = sorted(per.values())
    rows.setdefault(int(m), {})[c] = statistics.median(v) if v else float("nan")
print("mask   2xFETCH B/env   WRITE B/env   (stepw_kernel, 4096 envs, median over dispatches)")
for m in sorted(rows):
    r = rows[m]
    print(f"{m:5d}   {2 * r.get('FETCH_SIZE', float('nan')) * 1024 / 4096:13.1f}   {r.get('WRITE_SIZE', float('nan')) * 1024 / 4096:11.1f}")
PY
