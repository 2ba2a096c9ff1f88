#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration on stepw_kernel's access pattern (tools/fetch_calib.hip, built
# here: hipcc --offload-arch=gfx950 -O3 tools/fetch_calib.hip -o tools/fetch_calib), beside the
# config-2 kernel itself in the same session; then the raw TCC read-request split (64-B vs 32-B).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/fetch_calib; mkdir -p $O; export TMPDIR=/tmp
C2="--no-cpu-baseline --steps 10 --warmup 2 --settle 10 --policy-steps 0 --torch-policy-steps 0 --board-steps 0 --rollout-steps 0 --cold-steps 0 --config2-steps 200 --config4-steps 0 --large-steps 0 --from-reset-steps 0 --blocks-launches 0"
for c in FETCH_SIZE WRITE_SIZE "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"; do
  n=${c%% *}
  for mode in 0 1 2 3 4 5 6 7; do
    timeout -s KILL 60 rocprofv3 --pmc $c --output-format csv -d $O/calib_${n}_$mode -o run -- ./tools/fetch_calib 4096 200 $mode > $O/calib_${n}_$mode.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "calib $n mode $mode rc=$rc"; tail -5 $O/calib_${n}_$mode.log; exit $rc; }
  done
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O/c2_$n -o run -- python3 bench.py $C2 > $O/c2_$n.log 2>&1
  rc=$?; echo "config2 $n rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/c2_$n.log; exit $rc; }
done
python3 - $O <<'PY'
import csv, glob, os, re, statistics, sys, collections
O = sys.argv[1]
known = {"rd<0, 0>": 118, "rd<0, 1>": 118, "rd<1, 0>": 6, "rd<2, 0>": 88, "rd<3, 0>": 24, "rd<4, 0>": 118,
         "wr<0>": 83, "wr<1>": 29, "stepw_kernel<5, 13, 5, 8>": None}
res = collections.defaultdict(dict)
for f in glob.glob(f"{O}/*/**/*counter_collection.csv", recursive=True):
    per = collections.defaultdict(float)
    names = {}
    for r in csv.DictReader(open(f)):
        k = next((k for k in known if k in r["Kernel_Name"]), None)
        if k is None:
            continue
        per[(k, r["Counter_Name"], int(r["Dispatch_Id"]))] += float(r["Counter_Value"])
    agg = collections.defaultdict(list)
    for (k, c, d), v in per.items():
        agg[(k, c)].append(v)
    for (k, c), v in agg.items():
        res[k][c] = statistics.mean(v)
N = 4096
print(f"{'kernel':28s} {'known B/env':>11s} {'FETCH kB':>9s} {'2xFETCH B/env':>13s} {'WRITE B/env':>11s} {'RDREQ':>8s} {'RDREQ_32B':>9s}")
for k, b in known.items():
    r = res.get(k, {})
    fe, wr = r.get("FETCH_SIZE"), r.get("WRITE_SIZE")
    print(f"{k:28s} {str(b):>11s} {fe if fe is None else round(fe, 1)!s:>9s} "
          f"{'' if fe is None else round(2 * fe * 1024 / N, 1)!s:>13s} {'' if wr is None else round(wr * 1024 / N, 1)!s:>11s} "
          f"{r.get('TCC_EA0_RDREQ_sum', '')!s:>8s} {r.get('TCC_EA0_RDREQ_32B_sum', '')!s:>9s}")
PY
