"""Per-phase cycles per wave-step of the createBoard kernels (65 536 envs, 6 statics, random moves,
autoreset) on a -DBE_DIAG_STAMPS build (BALLENV_LIB=tools/diag/st/libballenv.so).
Phases: 0 state loads, 1 move + distances + collisions + reward + per-step stores, 2 autoreset
(wave-cooperative Philox resets), 3 features, 4 feature copy-out."""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import gym_ballenv_amd as gb  # noqa: E402

N, T = 65536, 100
b = gb.BatchedBoard(N, 6, device="cuda:0", seed=0xB0A2D, autoreset=True, time_limit=1000)
lib = b._lib
lib.be_board_diag_stamps.argtypes = [C.c_void_p]
b.reset()
acts = torch.randint(0, 4, (T, N), dtype=torch.uint8, device="cuda:0")
for name, fn in (("be_board_step (last of 100 launches)", lambda: [b.step(acts[t]) for t in range(T)]),
                 ("be_board_rollout (100 steps, one launch)", lambda: b.rollout(acts))):
    fn()
    fn()
    torch.cuda.synchronize()
    cy = np.zeros((1 << 14, 8), np.uint64)
    assert lib.be_board_diag_stamps(cy.ctypes.data_as(C.c_void_p)) == 0
    steps = 1 if "step (" in name else T
    ph = cy[:N // 64].astype(np.float64) / steps
    tot = ph.sum(1)
    print(f"{name}: cycles per wave-step p50 {np.median(tot):.0f} p90 {np.percentile(tot, 90):.0f} max {tot.max():.0f}")
    for k in range(5):
        print(f"  phase {k}: p50 {np.median(ph[:, k]):7.0f}  p90 {np.percentile(ph[:, k], 90):7.0f}  max {ph[:, k].max():7.0f}")
    if steps == 1:   # slots 5 / 6: the wave's finished envs / those left to the general passes
        nf, fb = cy[:N // 64, 5].astype(int), cy[:N // 64, 6].astype(int)
        for v in sorted(set(nf.tolist())):
            w = nf == v
            print(f"  waves with {v} resets: {w.sum():4d}, phase 2 p50 {np.median(ph[w, 2]):6.0f} max {ph[w, 2].max():6.0f},"
                  f" total p50 {np.median(tot[w]):6.0f} max {tot[w].max():6.0f}, general-pass envs {fb[w].sum()}")
b.close()
