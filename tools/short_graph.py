"""Why a 20-step timed region runs slower per kernel than a long one.  65 536 envs, W=10, graphs of
20 step launches, each replay timed alone with HIP events after a synchronize (as bench.py does):

  cyclic : bench.py's short command -- the same 20 action rows replayed over and over
           (settle + timed region), so each env repeats a 20-step action cycle;
  fresh  : a new 20-row block of random actions for every replay;
  b2b    : cyclic, but the timed replays follow each other with no synchronize in between;
  span   : cyclic, back to back, one event pair around all the timed replays.

    python tools/short_graph.py
"""
import ctypes as C
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import gym_ballenv_amd as gb  # noqa: E402
from gym_ballenv_amd import _abi  # noqa: E402

N, W = 65536, 10
K = int(os.environ.get("K", 20))          # launches per graph
G = 1200 // K
dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
lib = _abi.lib()


def graphs_for(env, acts, blocks):
    out = []
    cap = torch.cuda.Stream(dev)
    for b in blocks:
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=cap):
            cs = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
            for t in range(b * K, b * K + K):
                assert lib.be_step(env._ctx, C.byref(env._st), C.c_void_p(acts[t].data_ptr()), None, None,
                                   C.byref(env._out), cs) == 0
        out.append(g)
    torch.cuda.synchronize(dev)
    return out


def run(kind):
    env = gb.BatchedBallEnv(N, W, gb.EnvConfig(), device=dev, seed=0xBA11)
    acts = env.sample_actions(K * G, seed=0xBA11)
    gs = graphs_for(env, acts, range(G) if kind == "fresh" else [0])
    env.reset()
    stream = torch.cuda.current_stream(dev)
    seq = [gs[i % len(gs)] for i in range(G)]
    for g in seq[:G // 3]:      # settle: 400 steps
        g.replay()
    torch.cuda.synchronize(dev)
    us = []
    evs = []
    if kind == "span":          # one event pair around all the timed replays
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for g in seq[G // 3:]:
            g.replay()
        e1.record(stream)
        torch.cuda.synchronize(dev)
        n = (G - G // 3) * K
        print(f"span    us/step over {n} steps in {K}-step replays: {e0.elapsed_time(e1) * 1e3 / n:.3f}", flush=True)
        env.close()
        return
    for g in seq[G // 3:]:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        if kind != "b2b":
            torch.cuda.synchronize(dev)
        e0.record(stream)
        g.replay()
        e1.record(stream)
        evs.append((e0, e1))
    torch.cuda.synchronize(dev)
    us = [a.elapsed_time(b) * 1e3 / K for a, b in evs]
    print(f"{kind:7s} us/step per %d-step replay" % K + f": median {statistics.median(us):.3f}  min {min(us):.3f}  "
          f"max {max(us):.3f}  (steps 400..{G * K})", flush=True)
    env.close()


for kind in os.environ.get("KINDS", "cyclic fresh b2b cyclic").split():
    run(kind)
