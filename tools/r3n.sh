set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r3n
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r3n/pytest_gpu.log 2>&1
rc=$?; tail -2 gpurun_out/r3n/pytest_gpu.log; [ $rc -ne 0 ] && { grep -E "FAIL|^E " gpurun_out/r3n/pytest_gpu.log | head -20; exit $rc; }
# rocprofv3 of the default bench command (the driver's N=1 form)
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3n/prof_default -o run -- python3 bench.py > gpurun_out/r3n/bench_default_rocprof.log 2>&1
rc=$?; tail -c 300 gpurun_out/r3n/bench_default_rocprof.log; echo; exit $rc
