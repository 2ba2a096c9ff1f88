"""In-tree build of libballenv.so (gfx950) -- also run by __graft_entry__.build().

    python -m gym_ballenv_amd.build [--force]
"""
from __future__ import annotations

import os
import subprocess
import sys

PKG = os.path.dirname(os.path.realpath(__file__))
ROOT = os.path.dirname(PKG)
SRC = os.path.join(PKG, "csrc", "ballenv.hip")
DEPS = [os.path.join(PKG, "csrc", "policy.hip")]
HDR = os.path.join(ROOT, "include", "ballenv.h")
OUT = os.path.join(PKG, "libballenv.so")
ARCH = os.environ.get("BALLENV_OFFLOAD_ARCH", "gfx950")

HIPCC_FLAGS = ["-O3", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off", "-fno-fast-math",
               f"--offload-arch={ARCH}"]


def _stale(out, deps):
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(d) > t for d in deps)


def build_library(force: bool = False, verbose: bool = True) -> str:
    if force or _stale(OUT, [SRC, HDR, __file__, *DEPS]):
        hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
        cmd = [hipcc, *HIPCC_FLAGS, "-I", os.path.join(ROOT, "include"), SRC, "-o", OUT + ".tmp"]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
        os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    build_library(force="--force" in sys.argv)
