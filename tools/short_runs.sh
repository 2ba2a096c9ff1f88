#!/bin/bash
# Headline step leg only, at the driver's short command (--steps 20 --warmup 5) and at 1000 steps,
# for each launch mode; then a kernel trace of the short graph run (gaps between launches).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/short; export TMPDIR=/tmp
LEGS="--no-cpu-baseline --policy-steps 0 --board-steps 0 --rollout-steps 0"
for mode in ${MODES:-graph loop}; do
  for sw in "20 5" "1000 100"; do
    set -- $sw
    timeout -k 10 120 python3 bench.py $LEGS --mode $mode --steps $1 --warmup $2 > gpurun_out/short/$mode-$1.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "$mode $1 rc=$rc"; tail -5 gpurun_out/short/$mode-$1.log; exit $rc; }
    python3 -c "
import json; d = json.loads(open('gpurun_out/short/$mode-$1.log').read().strip().splitlines()[-1])
print('%-6s K=%-5s value %.3e  wall us/step %.3f  event us/step %.3f' % ('$mode', '$1', d['value'], d['ms_per_step'] * 1e3, d['roofline']['kernel_us_mean']))"
  done
done
if [ "${TRACE:-1}" = "1" ]; then
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/short/trace -o run -- \
      python3 bench.py $LEGS --mode graph --steps 20 --warmup 5 > gpurun_out/short/trace.log 2>&1 || exit $?
  python3 - <<'EOF'
import csv, glob
f = glob.glob("gpurun_out/short/trace/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
rows = [r for r in rows if "step2_kernel" in r["Kernel_Name"] or "be_kernel" in r["Kernel_Name"]]
prev = None
for r in rows[-45:]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print("dur %6.2f us  gap %8.2f us" % ((e - s) / 1e3, (s - prev) / 1e3 if prev else 0.0))
    prev = e
EOF
fi
