"""Step the 65 536-env batch as S sub-batches on S HIP streams (envs are independent, Philox keys
are global env ids, so the trajectories are the same as one batch's).  Times K graph-replayed
steps three ways: one kernel per step (S=1); S kernels per step forked from and joined back to
the main stream every step; S independent chains joined only at the end of the K steps.

    python tools/split_streams.py [K]
"""
import ctypes as C
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import gym_ballenv_amd as gb  # noqa: E402
from gym_ballenv_amd import _abi  # noqa: E402

N, W = 65536, 10
K = int(sys.argv[1]) if len(sys.argv) > 1 else 200
dev = torch.device("cuda:0")
lib = _abi.lib()


def make(S):
    envs = [gb.BatchedBallEnv(N // S, W, gb.EnvConfig(), device=dev, seed=0xBA11, env_offset=s * (N // S))
            for s in range(S)]
    acts = [e.sample_actions(K, seed=0xBA11) for e in envs]
    for e in envs:
        e.reset()
    return envs, acts


def launch(e, a, t, stream):
    rc = lib.be_step(e._ctx, C.byref(e._st), C.c_void_p(a[t].data_ptr()), None, None, C.byref(e._out),
                     C.c_void_p(stream.cuda_stream))
    assert rc == 0


def capture(S, mode):
    envs, acts = make(S)
    main = torch.cuda.Stream(dev)
    side = [torch.cuda.Stream(dev) for _ in range(S)]
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=main):
        cur = torch.cuda.current_stream(dev)
        if S == 1:
            for t in range(K):
                launch(envs[0], acts[0], t, cur)
        elif mode == "join":
            for t in range(K):
                fork = torch.cuda.Event()
                fork.record(cur)
                done = []
                for s in range(S):
                    side[s].wait_event(fork)
                    launch(envs[s], acts[s], t, side[s])
                    ev = torch.cuda.Event()
                    ev.record(side[s])
                    done.append(ev)
                for ev in done:
                    cur.wait_event(ev)
        else:   # independent chains, joined at the end
            fork = torch.cuda.Event()
            fork.record(cur)
            done = []
            for s in range(S):
                side[s].wait_event(fork)
                for t in range(K):
                    launch(envs[s], acts[s], t, side[s])
                ev = torch.cuda.Event()
                ev.record(side[s])
                done.append(ev)
            for ev in done:
                cur.wait_event(ev)
    return g, envs


def timeit(g):
    g.replay()
    torch.cuda.synchronize(dev)
    best = []
    for _ in range(5):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        g.replay()
        torch.cuda.synchronize(dev)
        best.append(time.perf_counter() - t0)
    return min(best) / K * 1e6


for S, mode in ((1, "-"), (2, "join"), (2, "chains"), (4, "join"), (4, "chains")):
    g, envs = capture(S, mode)
    us = timeit(g)
    print(f"S={S} {mode:6s}: {us:6.2f} us per 65536-env step = {N / us * 1e-3:.3f}e9 env-steps/s", flush=True)
    del g
    for e in envs:
        e.close()
