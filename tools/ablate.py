"""Kernel-time ablation (diagnostics): be_step duration per phase-skip mask and batch size.

Each config gets its own context (BALLENV_DEBUG_SKIP is read at be_create);
all run interleaved in one process (rule: A/B in one process), HIP events
around each launch, median of rounds.
"""
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import gym_ballenv_amd as gb  # noqa: E402
from gym_ballenv_amd import _abi  # noqa: E402


def make(n, w, dbg, lpe=""):
    os.environ["BALLENV_DEBUG_SKIP"] = str(dbg)
    if lpe:
        os.environ["BALLENV_STEP_LPE"] = lpe
    ns, nd = (int(x) for x in os.environ.get("OBST", "13,5").split(","))   # static, dynamic obstacles
    env = gb.BatchedBallEnv(n, w, gb.EnvConfig(num_static=ns, num_dynamic=nd), device="cuda:0", seed=1)
    os.environ.pop("BALLENV_DEBUG_SKIP")
    os.environ.pop("BALLENV_STEP_LPE", None)
    env.reset()
    acts = env.sample_actions(64, seed=2)
    return env, acts


def time_env(env, acts, launches=100):
    lib = _abi.lib()
    s = torch.cuda.current_stream()
    sp = C.c_void_p(s.cuda_stream)
    st, out = C.byref(env._st), C.byref(env._out)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(launches)]
    for t in range(launches):
        ev[t][0].record(s)
        lib.be_step(env._ctx, st, C.c_void_p(acts.data_ptr() + (t % 64) * env.num_envs), None, None, out, sp)
        ev[t][1].record(s)
    torch.cuda.synchronize()
    d = sorted(a.elapsed_time(b) * 1e3 for a, b in ev)
    return d[len(d) // 2]


def time_graph(env, acts, launches=200):
    """Per-launch time of `launches` back-to-back be_step launches replayed from one HIP graph
    (the bench's launch mode), events around the replay."""
    lib = _abi.lib()
    st, out = C.byref(env._st), C.byref(env._out)
    if not hasattr(env, "_abl_graph"):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=torch.cuda.Stream()):
            sp = C.c_void_p(torch.cuda.current_stream().cuda_stream)
            for t in range(launches):
                lib.be_step(env._ctx, st, C.c_void_p(acts.data_ptr() + (t % 64) * env.num_envs), None, None, out, sp)
        env._abl_graph = g
        g.replay()
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record(s)
    env._abl_graph.replay()
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / launches


def main():
    masks = [int(m, 0) for m in os.environ.get("MASKS", "0,1,2,6,8,16,24,32,63").split(",")]
    sizes = [int(n) for n in os.environ.get("SIZES", "65536,262144,1048576").split(",")]
    W = int(os.environ.get("W", "10"))
    lpes = os.environ.get("LPES", "").split(",")     # BALLENV_STEP_LPE per context ("" = dispatch)
    envs = {(n, m, l): make(n, W, m, l) for n in sizes for m in masks for l in lpes}
    res = {k: [] for k in envs}
    for _ in range(5):
        for k, (e, a) in envs.items():
            res[k].append(time_graph(e, a) if os.environ.get("GRAPH") else time_env(e, a))
    for (n, m, l), v in sorted(res.items()):
        v.sort()
        print(json.dumps({"envs": n, "mask": m, "lpe": l, "kernel": envs[(n, m, l)][0].kernel_name("step"), "us_median": round(v[len(v) // 2], 2), "us_min": round(v[0], 2),
                          "ns_per_env": round(v[len(v) // 2] * 1e3 / n, 3)}))


if __name__ == "__main__":
    main()
