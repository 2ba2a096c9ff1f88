#!/bin/bash
# Per-wave phase stamps of the step kernel (tools/stamps.hip on the -DBE_DIAG_STAMPS library),
# for the two fixed-shape step kernels (BALLENV_STEP_LPE=1: be_kernel<10,0,13,5>; 2: step2_kernel).
# Build here first: BUILD=1 bash tools/stamps_run.sh (no GPU needed).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
F="-O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math --offload-arch=gfx950 -I include -I gym-ballenv_amd/csrc"
ST=${ST:-diag/st}   # under tools/ (tools/diag is not pushed to the box: ST=stlib for a box run, deleted after)
if [ "${BUILD:-0}" = "1" ]; then
  mkdir -p tools/$ST
  /opt/rocm/bin/hipcc $F -shared -DBE_DIAG_STAMPS gym-ballenv_amd/csrc/ballenv.hip gym-ballenv_amd/csrc/policy.hip \
      gym-ballenv_amd/csrc/features.hip gym-ballenv_amd/csrc/board.hip -o tools/$ST/libballenv.so || exit 1
  /opt/rocm/bin/hipcc $F tools/stamps.hip -Ltools/$ST -lballenv -Wl,-rpath,"\$ORIGIN/$ST" -o tools/stamps || exit 1
  echo built; exit 0
fi
mkdir -p gpurun_out
for L in ${LPES:-1 2}; do
  BALLENV_STEP_LPE=$L timeout -k 10 120 ./tools/stamps ${N:-65536} > gpurun_out/stamps_lpe${L}_${N:-65536}${TAG:-}.txt 2>&1
  rc=$?; echo "stamps LPE=$L rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/stamps_lpe${L}_${N:-65536}${TAG:-}.txt; exit $rc; }
done
exit 0
