set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_bench_contract.py > gpurun_out/r3k_pytest.log 2>&1
rc=$?; grep -E "PASS|FAIL" gpurun_out/r3k_pytest.log; tail -3 gpurun_out/r3k_pytest.log; exit $rc
