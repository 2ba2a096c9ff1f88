#!/bin/bash
# Step-kernel time per library variant (VARIANTS="base ct128 ..."; base = the in-tree build, others
# tools/diag/<name>/libballenv.so from build_ab_lib.sh) at ENVS / W / LANES through lane_sweep.py,
# then (BENCH=1) the default bench line.  Every GPU step under its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${ROUND:-r04}_blocks; mkdir -p $O
for v in ${VARIANTS:-base}; do
  lib=""; [ "$v" != base ] && lib=tools/diag/$v/libballenv.so
  BALLENV_LIB=$lib timeout -k 10 200 python -u tools/lane_sweep.py --window ${W:-10} --envs ${ENVS:-32768,65536} \
      --lanes ${LANES:-2} --reps ${REPS:-2} ${SWEEP_ARGS:-} > $O/sweep_${TAG:-w${W:-10}}_$v.jsonl 2>&1 || exit $?
done
if [ "${BENCH:-0}" = "1" ]; then
  timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
fi
