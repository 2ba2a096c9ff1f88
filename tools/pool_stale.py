"""How often a finishing env finds its autoreset-pool entry stale, per refill period (CPU, oracle).

The pool holds per env the resets into episodes e+1 and e+2, e = the env's episode at
the last fill; a fill runs at reset and every `period` be_step calls.  An env finishing its third
episode since that fill finds no current entry and draws its reset inline -- and one such env makes
its wave (32 envs of step2_kernel, 64 lanes) as slow as a wave without the pool, which can set the
launch's tail.  This replays the same Philox trajectories as the GPU (the oracle is bit-exact with
the step kernels) and counts, per period, the stale finishes per step and the fraction of launches
with at least one stale wave.

    python tools/pool_stale.py [envs] [steps] [periods...]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gym_ballenv_amd import _abi  # noqa: E402
from gym_ballenv_amd.config import EnvConfig  # noqa: E402
from oracle import oracle  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
T = int(sys.argv[2]) if len(sys.argv) > 2 else 1400
PERIODS = [int(p) for p in sys.argv[3:]] or [16, 32, 64, 128, 512]
SKIP = int(os.environ.get("SKIP", "400"))   # bench.py's settle: the timed region starts past the post-reset transient
EPW = 32            # envs per wave of step2_kernel (W=10)

cfg = EnvConfig().to_abi(N, 10, 0, 0xBA11)
st, out = oracle.new_state(cfg), oracle.new_out(cfg)
oracle.reset(cfg, st, out)
acts = oracle.sample_actions(cfg, T, seed=1)
fin = np.zeros((T, N), bool)
for t in range(T):
    oracle.step(cfg, st, out, actions=acts[t])
    fin[t] = out["done"] != 0
print(f"{N} envs, {T} steps; finishes per step after {SKIP}: {fin[SKIP:].sum(1).mean():.1f}", flush=True)
for P in PERIODS:
    since = np.zeros(N, np.int32)          # finishes since the last fill (fill at reset: step 0)
    stale_per_step, launches_stale, waves_stale = [], 0, []
    for t in range(T):
        if t > 0 and t % P == 0:
            since[:] = 0                   # a fill queued before launch t refreshes every entry
        f = fin[t]
        since[f] += 1
        stale = f & (since > 2)
        if t >= SKIP:
            stale_per_step.append(stale.sum())
            w = np.unique(np.nonzero(stale)[0] // EPW).size
            waves_stale.append(w)
            launches_stale += w > 0
    n = T - SKIP
    print(f"period {P:5d}: stale finishes per step {np.mean(stale_per_step):.3f}, launches with a stale wave "
          f"{launches_stale / n:.3f}, stale waves per launch {np.mean(waves_stale):.3f}", flush=True)
