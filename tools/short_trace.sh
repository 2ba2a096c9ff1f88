#!/bin/bash
# Kernel trace of back-to-back K-launch graph replays (tools/short_graph.py b2b): step-kernel
# duration by position inside the graph, for K = 20 and 100.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/strace; export TMPDIR=/tmp
for K in ${KS:-20 100}; do
  K=$K KINDS="fresh b2b" timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/strace/k$K -o run -- \
      python3 tools/short_graph.py > gpurun_out/strace/k$K.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "K=$K rc=$rc"; tail -5 gpurun_out/strace/k$K.log; exit $rc; }
  cat gpurun_out/strace/k$K.log | grep us/step
  python3 - $K <<'PY'
import csv, glob, statistics, sys
K = int(sys.argv[1])
f = glob.glob(f"gpurun_out/strace/k{K}/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
rows = [r for r in rows if "step2_kernel" in r["Kernel_Name"]]
# the last run (b2b) : its timed replays are the last 2/3 of its 1200 launches
rows = rows[-800:]
pos = [[] for _ in range(K)]
gaps = [[] for _ in range(K)]
prev = None
for i, r in enumerate(rows):
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    pos[i % K].append((e - s) / 1e3)
    if prev is not None:
        gaps[i % K].append((s - prev) / 1e3)
    prev = e
span = (int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])) / 1e3 / len(rows)
print(f"K={K}: span per launch {span:.3f} us; median duration by position in the graph:")
for k in list(range(min(K, 6))) + [K - 2, K - 1]:
    print(f"  pos {k:3d}: dur {statistics.median(pos[k]):6.2f}  gap before {statistics.median(gaps[k]) if gaps[k] else 0:6.2f} us")
PY
done
