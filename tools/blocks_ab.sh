#!/bin/bash
# prep_state2 block counts (bench.py's blocks_obs leg): feature / bench-contract GPU tests, then the
# in-tree library against tools/diag/$B, interleaved twice.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/blk_ab; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_features_golden.py tests/test_bench_contract.py -m gpu -x -q -p no:cacheprovider \
    --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
ARGS="--no-cpu-baseline --steps 10 --warmup 2 --settle 10 --policy-steps 0 --torch-policy-steps 0 --board-steps 0 --rollout-steps 0 --cold-steps 0 --config2-steps 0 --large-steps 0 --from-reset-steps 0 --blocks-launches 200"
for r in 1 2; do
  for v in new ${B:-old}; do   # B: one or more A/B builds
    if [ $v = new ]; then L=""; else L=tools/diag/$v/libballenv.so; fi
    BALLENV_LIB=$L timeout -k 10 200 python3 bench.py $ARGS > $O/$v.$r.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "$v rc=$rc"; tail -5 $O/$v.$r.log; exit $rc; }
    python3 -c "
import json; d = json.loads(open('$O/$v.$r.log').read().strip().splitlines()[-1])['blocks_obs']
print('%-4s r$r' % '$v', '  '.join('%s %s %.2f us (%.2f)' % (n[5:], k, d[n][k]['kernel_us_mean'], d[n][k]['roofline']['frac']) for n in d if n.startswith('envs') for k in ('u8', 'f32')))"
  done
done
