#!/bin/bash
# Diagnostic builds (git-ignored): libballenv variants with lanes-per-env 1/2/4 under
# tools/diag/lpeN/ and a microbench binary per variant (tools/mb_lpeN, RUNPATH -> its lib).
set -eu
cd "$(dirname "$0")/.."
F="-O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math --offload-arch=gfx950 -I include"
for L in ${LPES:-1 2 4}; do
  mkdir -p tools/diag/lpe$L
  /opt/rocm/bin/hipcc $F -shared -DBE_LPE=$L gym-ballenv_amd/csrc/ballenv.hip -o tools/diag/lpe$L/libballenv.so &
done
wait
for L in ${LPES:-1 2 4}; do
  /opt/rocm/bin/hipcc $F tools/microbench.hip -Ltools/diag/lpe$L -lballenv -Wl,-rpath,'$ORIGIN/diag/lpe'$L -o tools/mb_lpe$L &
done
wait
echo built
# per-wave phase stamps (-DBE_DIAG_STAMPS) for LPE 1 and 2
if [ "${STAMPS:-1}" = "1" ]; then
  for L in 1 2; do
    mkdir -p tools/diag/st$L
    /opt/rocm/bin/hipcc $F -shared -DBE_LPE=$L -DBE_DIAG_STAMPS gym-ballenv_amd/csrc/ballenv.hip -o tools/diag/st$L/libballenv.so &
  done
  wait
  for L in 1 2; do
    /opt/rocm/bin/hipcc $F tools/stamps.hip -Ltools/diag/st$L -lballenv -Wl,-rpath,'$ORIGIN/diag/st'$L -o tools/stamps_lpe$L &
  done
  wait
  echo built stamps
fi
