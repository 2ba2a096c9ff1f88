"""Per-phase cycles per wave-step of the small-batch fused rollout (rolloutw_kernel) against the
one-lane rollout_kernel, W=5, on a -DBE_DIAG_STAMPS build (BALLENV_LIB=tools/diag/st/libballenv.so).
rolloutw phases: 0 counter + Philox + dynamic moves, 1 agent move + f64 distance / reward term,
2 obstacle tests + group OR, 3 reward/done + per-step stores + stats record, 4 autoreset,
5 obs stage + copy-out, 6 stats fold (every 32 steps) + action hand-over.
rollout_kernel phases (PH in its body): 4 action load, 5 physics, 6 autoreset, 7 raster + stage."""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import gym_ballenv_amd as gb  # noqa: E402
from gym_ballenv_amd import _abi  # noqa: E402

DW, DP = 1 << 16, 16
lib = _abi.lib()
lib.be_diag_stamps.argtypes = [C.c_void_p, C.c_void_p]
N, W, T = int(os.environ.get("N", "4096")), 5, 100
for lpe in ("8", "1"):
    os.environ["BALLENV_ROLLOUT5_LPE"] = lpe
    env = gb.BatchedBallEnv(N, W, gb.EnvConfig(), device="cuda:0", seed=0xBA11)
    acts = env.sample_actions(T, seed=3)
    env.reset()
    for _ in range(3):
        env.rollout(acts)
    torch.cuda.synchronize()
    rt = np.zeros((DW, DP), np.uint64)
    cy = np.zeros((DW, DP), np.uint64)
    assert lib.be_diag_stamps(rt.ctypes.data_as(C.c_void_p), cy.ctypes.data_as(C.c_void_p)) == 0
    waves = N * int(lpe) // 64
    ph = cy[:waves, :8].astype(np.float64) / T
    print(f"{env.kernel_name('rollout')}: {N} envs, {waves} waves; cycles per wave-step: total p50 {np.median(ph.sum(1)):.0f}")
    for k in range(8):
        print(f"  phase {k}: p50 {np.median(ph[:, k]):7.0f}  p90 {np.percentile(ph[:, k], 90):7.0f}")
    env.close()

# stepw_kernel (one step per launch): phases 0 prologue + loads + barrier, 1 counter + Philox +
# dynamic moves, 2 agent move + f64 distance / reward term, 3 obstacle tests + group OR,
# 4 reward/done + state stores + stats (barrier, wave-0 fold), 5 terminal obs + autoreset,
# 6 obs stage + copy-out; the last of 50 back-to-back launches
os.environ["BALLENV_STEP5_LPE"] = "8"
env = gb.BatchedBallEnv(N, W, gb.EnvConfig(), device="cuda:0", seed=0xBA11)
acts = env.sample_actions(50, seed=3)
env.reset()
for t in range(50):
    env.step(acts[t])
torch.cuda.synchronize()
rt = np.zeros((DW, DP), np.uint64)
cy = np.zeros((DW, DP), np.uint64)
assert lib.be_diag_stamps(rt.ctypes.data_as(C.c_void_p), cy.ctypes.data_as(C.c_void_p)) == 0
waves = N * 8 // 64
ph = cy[:waves, :8].astype(np.float64)
print(f"{env.kernel_name('step')}: {N} envs, {waves} waves; cycles per wave (one launch): total p50 {np.median(ph.sum(1)):.0f} p90 {np.percentile(ph.sum(1), 90):.0f}")
for k in range(7):
    print(f"  phase {k}: p50 {np.median(ph[:, k]):7.0f}  p90 {np.percentile(ph[:, k], 90):7.0f}")
env.close()
