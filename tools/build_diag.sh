#!/bin/bash
# Diagnostics builds (git-ignored; csrc/diag.h): the whole library with -DBE_DIAG_STAMPS (per-wave
# phase stamps + the DBG skip bits) under tools/diag/st/, and the C harnesses linked against it:
# tools/stamps (per-wave stamps of the step kernel) and tools/microbench (memory floors, launches).
set -eu
cd "$(dirname "$0")/.."
F="-O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math --offload-arch=gfx950 -I include"
bash tools/build_ab_lib.sh st -DBE_DIAG_STAMPS
/opt/rocm/bin/hipcc $F tools/stamps.hip -Ltools/diag/st -lballenv -Wl,-rpath,'$ORIGIN/diag/st' -o tools/stamps &
/opt/rocm/bin/hipcc $F tools/microbench.hip -Lgym-ballenv_amd -lballenv -Wl,-rpath,'$ORIGIN/../gym-ballenv_amd' -o tools/microbench &
wait
echo built tools/diag/st/libballenv.so tools/stamps tools/microbench
