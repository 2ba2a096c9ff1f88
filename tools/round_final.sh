#!/bin/bash
# A round's closing run (ROUND=r04 names the output dir): the full GPU suite and smoke, the driver's bench commands, and a rocprofv3
# kernel trace of the default bench command with its per-region summary (tools/trace_regions.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${ROUND:-r04}_final; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -ne 0 ] && { grep -E "^E |FAIL" $O/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.log 2>&1 || { tail -5 $O/bench_driver.log; exit 1; }
timeout -k 10 400 python bench.py > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
tail -c 400 $O/bench.log; echo
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_default -o run -- python3 bench.py > $O/bench_rocprof.log 2>&1 || { tail -5 $O/bench_rocprof.log; exit 1; }
python tools/trace_regions.py $(find $O/prof_default -name "*kernel_trace.csv" | head -1) > $O/regions.txt; cat $O/regions.txt
find $O/prof_default -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
rm -f $(find $O/prof_default -name "*kernel_trace.csv")
