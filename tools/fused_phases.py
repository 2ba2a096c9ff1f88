"""Per-phase cycles of the fused rollout kernels (diagnostics build -DBE_DIAG_STAMPS: each wave
accumulates s_memtime deltas per phase over a launch's steps, PH() in csrc/ballenv.hip).

    BALLENV_LIB=tools/diag/st/libballenv.so python tools/fused_phases.py
Phases (policy rollout): 0 uniform + list append, 1 barrier 1, 2 dense tiles, 3 barrier 2,
4 logits + softmax/draw + action stores, 5 physics (move ... reward/done stores, stats),
6 autoreset, 7 raster + stage (+ recorded obs).  The random-action rollout has 4..7 only.
"""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import gym_ballenv_amd as gb  # noqa: E402
from gym_ballenv_amd import _abi  # noqa: E402
from gym_ballenv_amd.policy import Policy, reference_weights  # noqa: E402

NAMES = ["uniform+list", "barrier1", "tiles", "barrier2", "logits+draw", "physics", "reset", "raster+stage"]
DW, DP = 1 << 16, 16


def read(lib, waves, steps):
    rt = np.zeros((DW, DP), np.uint64)
    cy = np.zeros((DW, DP), np.uint64)
    assert lib.be_diag_stamps(rt.ctypes.data_as(C.c_void_p), cy.ctypes.data_as(C.c_void_p)) == 0
    ph = cy[:waves, :8].astype(np.float64) / steps
    tot = ph.sum(1)
    print(f"  cycles per wave-step: total p50 {np.median(tot):.0f} (p90 {np.percentile(tot, 90):.0f})")
    for k, n in enumerate(NAMES):
        print(f"    {k} {n:14s} p50 {np.median(ph[:, k]):7.0f}  mean {ph[:, k].mean():7.0f}  p90 {np.percentile(ph[:, k], 90):7.0f}")


def main():
    lib = _abi.lib()
    lib.be_diag_stamps.argtypes = [C.c_void_p, C.c_void_p]
    dev = torch.device("cuda:0")
    N, W, T = 65536, 10, 100
    pol = Policy.from_npz(reference_weights(W), W)
    env = gb.BatchedBallEnv(N, W, gb.EnvConfig(), device=dev, seed=0xBA11)
    env.reset()
    ro = gb.Rollout(env, pol, horizon=T, backend="fused", chunk=T)
    for _ in range(3):
        ro.run()
    torch.cuda.synchronize()
    print("fused policy rollout (be_policy_rollout), 65536 envs, W=10, last launch of 100 steps:")
    read(lib, N // 64, T)
    ro.close()
    env.close()
    env = gb.BatchedBallEnv(N, W, gb.EnvConfig(), device=dev, seed=0xBA11)
    acts = env.sample_actions(T, seed=3)
    env.reset()
    for _ in range(3):
        env.rollout(acts)
    torch.cuda.synchronize()
    print("fused random-action rollout (be_rollout), same envs:")
    read(lib, N // 64, T)
    env.close()


if __name__ == "__main__":
    main()
