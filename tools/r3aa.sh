# full GPU suite on the round-3 tree (board single-chain resets + write-through, stepw prologue,
# blocks load chunks), then the blocks store-policy A/B
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r3aa
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r3aa/pytest_gpu.log 2>&1
rc=$?; tail -2 gpurun_out/r3aa/pytest_gpu.log; [ $rc -ne 0 ] && { grep -E "^E |FAIL" gpurun_out/r3aa/pytest_gpu.log | head -20; exit $rc; }
B="featnowt featold" bash tools/blocks_ab.sh
