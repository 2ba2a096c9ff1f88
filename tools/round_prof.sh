#!/bin/bash
# rocprofv3 kernel trace of the default bench command with its per-region summary, then the
# createBoard counters (the ROUND_pmc_board_step / _rollout profiles) and phase stamps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${ROUND:-r04}_prof; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_default -o run -- python3 bench.py > $O/bench_rocprof.log 2>&1 || { tail -5 $O/bench_rocprof.log; exit 1; }
python tools/trace_regions.py $O/prof_default/run_kernel_trace.csv > $O/regions.txt 2>&1; cat $O/regions.txt
tail -1 $O/bench_rocprof.log | cut -c1-200
gzip -f $O/prof_default/run_kernel_trace.csv
BALLENV_LIB=tools/diag/st/libballenv.so timeout -k 10 200 python tools/board_phases.py > $O/board_phases.txt 2>&1
grep -v amdgpu.ids $O/board_phases.txt
timeout -k 10 900 bash tools/pmc_passes.sh ${ROUND:-r04}_prof/pmc --no-cpu-baseline --steps 10 --warmup 2 --settle 10 \
    --policy-steps 0 --torch-policy-steps 0 --board-steps 200 --rollout-steps 0 --cold-steps 0 \
    --config2-steps 0 --large-steps 0 --from-reset-steps 0 --blocks-launches 0
rc=$?; echo "pmc rc=$rc"; [ $rc -ne 0 ] && exit $rc
python tools/pmc_report.py $O/pmc "board_kernel<6, false" 65536 --out $O/${ROUND:-r04}_pmc_board_step.json > /dev/null
python tools/pmc_report.py $O/pmc "board_kernel<6, true" 6553600 --out $O/${ROUND:-r04}_pmc_board_rollout.json > /dev/null
