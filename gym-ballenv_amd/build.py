"""In-tree build of libballenv.so (gfx950) -- also run by __graft_entry__.build().

    python -m gym_ballenv_amd.build [--force]

Two translation units, compiled separately (each embeds its own gfx950 code
object) and linked into one shared library:
  csrc/ballenv.hip  step / reset / observe kernels + the C ABI
  csrc/policy.hip   select_action kernel (-fno-slp-vectorize: scalar f32 FMAs
                    interleave better with MFMAs than SLP-packed ones on gfx950)
  csrc/features.hip sibling observation formats (prep_state2 block counts)
  csrc/board.hip    the createBoard physics profile + featureExtractor
"""
from __future__ import annotations

import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

PKG = os.path.dirname(os.path.realpath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
HDR = os.path.join(ROOT, "include", "ballenv.h")
OUT = os.path.join(PKG, "libballenv.so")
ARCH = os.environ.get("BALLENV_OFFLOAD_ARCH", "gfx950")

BASE_FLAGS = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-fast-math", f"--offload-arch={ARCH}"]
# -amdgpu-mfma-vgpr-form: MFMA accumulators in VGPRs.  The compiler's default put the fc1
# tiles' accumulators in AGPRs, which costs 12 v_accvgpr_read per tile row (of ~70 VALU); only
# the kernels with MFMAs (the policy forward and the fused policy rollouts) change.
VGPR_MFMA = ["-mllvm", "-amdgpu-mfma-vgpr-form"]
UNITS = {"ballenv.hip": VGPR_MFMA, "policy.hip": ["-fno-slp-vectorize", *VGPR_MFMA], "features.hip": [], "board.hip": []}
HEADERS = [HDR, *(os.path.join(CSRC, h) for h in ("philox.h", "internal.h", "policy_core.h", "diag.h"))]


def _stale(out, deps):
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(d) > t for d in deps)


def build_library(force: bool = False, verbose: bool = True, extra_flags=(), out: str = OUT) -> str:
    srcs = [os.path.join(CSRC, u) for u in UNITS]
    if not (force or extra_flags or _stale(out, [*srcs, *HEADERS, __file__])):
        return out
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    inc = ["-I", os.path.join(ROOT, "include"), "-I", CSRC]
    objs, cmds = [], []
    for u, flags in UNITS.items():
        obj = f"{out}.{os.path.splitext(u)[0]}.o"
        objs.append(obj)
        cmds.append([hipcc, *BASE_FLAGS, *flags, *extra_flags, *inc, "-c", os.path.join(CSRC, u), "-o", obj])

    def run(cmd):
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)

    with ThreadPoolExecutor(len(cmds)) as ex:
        list(ex.map(run, cmds))
    link = [hipcc, "-shared", f"--offload-arch={ARCH}", *objs, "-o", out + ".tmp"]
    run(link)
    os.replace(out + ".tmp", out)
    for o in objs:
        os.remove(o)
    return out


if __name__ == "__main__":
    build_library(force="--force" in sys.argv)
