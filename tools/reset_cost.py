"""What the autoreset pass costs a fixed-shape step launch, measured on the release library.

Three contexts per size, interleaved (graph-replayed be_step launches, HIP events, median of rounds),
statistics slots off in all (a done env's fold is not what is measured):
  reset   autoreset 1, TimeLimit 1000, ep_len spread uniformly over [0, 1000) first -- the steady state
          of a long run (~N/900 resets per step, 85 % of them truncations)
  coll    autoreset 1, no TimeLimit (collision / goal resets only)
  none    autoreset 0, no TimeLimit: no env is ever reset (done envs step on; no reset pass runs)
Outputs of `none` are a different trajectory, not wrong ones: it is the same kernel without resets.
usage: SIZES=32768,65536 python tools/reset_cost.py
"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import gym_ballenv_amd as gb  # noqa: E402
from gym_ballenv_amd import _abi  # noqa: E402


def make(n, autoreset, tl, spread):
    env = gb.BatchedBallEnv(n, 10, gb.EnvConfig(autoreset=autoreset, time_limit=tl), device="cuda:0", seed=3,
                            track_stats=False)
    env.reset()
    if spread:
        env.ep_len.copy_(torch.randint(0, 1000, (n,), dtype=torch.int32, device="cuda:0"))
    acts = env.sample_actions(200, seed=4)
    lib = _abi.lib()
    st, out = C.byref(env._st), C.byref(env._out)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=torch.cuda.Stream()):
        sp = C.c_void_p(torch.cuda.current_stream().cuda_stream)
        for t in range(200):
            lib.be_step(env._ctx, st, C.c_void_p(acts[t].data_ptr()), None, None, out, sp)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    env._keep_acts = acts      # the graph reads these rows: keep them alive
    return env, g


def timed(g, reps=5):
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        g.replay()
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / (reps * 200)


for n in [int(x) for x in os.environ.get("SIZES", "32768,65536").split(",")]:
    arms = {"reset": make(n, True, 1000, True), "coll": make(n, True, 0, False), "none": make(n, False, 0, False)}
    res = {k: [] for k in arms}
    for r in range(int(os.environ.get("ROUNDS", "5"))):
        for k, (env, g) in arms.items():
            res[k].append(timed(g))
    for k, v in res.items():
        v.sort()
        print(f"envs {n} {k:6s} kernel {arms[k][0].kernel_name('step')}: us per launch median {v[len(v) // 2]:.3f} "
              f"min {v[0]:.3f} max {v[-1]:.3f}", flush=True)
    for env, _ in arms.values():
        env.status()
        env.close()
