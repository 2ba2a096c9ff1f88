#!/bin/bash
# A/B of step-kernel builds on the headline leg: each arg "name@lib@VAR=val" runs bench.py's step leg
# (1000 graph-replayed steps) with BALLENV_LIB=lib (empty: the in-tree library) and the env setting,
# then the same command under rocprofv3 --kernel-trace --stats.  Results: gpurun_out/ab/<name>.*
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab; export TMPDIR=/tmp
ARGS="--no-cpu-baseline --steps ${STEPS:-1000} --warmup 100 --policy-steps 0 --board-steps 0 --rollout-steps 0 ${BENCH_ARGS:-}"
for spec in "$@"; do
  IFS=@ read -r name lib envset <<< "$spec"
  envs=(); [ -n "$lib" ] && envs+=("BALLENV_LIB=$lib"); [ -n "$envset" ] && envs+=("$envset")
  env "${envs[@]}" timeout -k 10 120 python3 bench.py $ARGS > gpurun_out/ab/$name.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "$name rc=$rc"; tail -5 gpurun_out/ab/$name.log; exit $rc; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab/$name.log').read().strip().splitlines()[-1]); r=d['roofline']; print('%-14s %s value %.3e  us/step %.3f  kernel_us %.3f  frac %.3f' % ('$name', r['kernel'], d['value'], d['ms_per_step']*1e3, r['kernel_us_mean'], r['frac']))"
  if [ "${PROF:-1}" = "1" ]; then
    for e in "${envs[@]}"; do export "$e"; done
    timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab/prof_$name -o run -- python3 bench.py $ARGS > gpurun_out/ab/prof_$name.log 2>&1
    rc=$?
    for e in "${envs[@]}"; do unset "${e%%=*}"; done
    [ $rc -ne 0 ] && { echo "prof $name rc=$rc"; exit $rc; }
    python3 - "$name" <<'PY'
import csv, glob, sys
n = sys.argv[1]
f = glob.glob(f"gpurun_out/ab/prof_{n}/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "step" in r["Name"] or "be_kernel" in r["Name"]:
        print(f"   rocprof {r['Name'][29:70]:42s} calls {r['Calls']:>5s} avg_us {float(r['AverageNs'])/1e3:7.3f} min {float(r['MinNs'])/1e3:7.3f}")
PY
  fi
done
exit 0
