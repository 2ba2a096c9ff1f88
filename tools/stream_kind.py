"""Short timed regions (K=20 graph-replayed step launches, 65 536 envs) on torch's default stream
against a separately created stream: wall and event time per region, median of 40."""
import ctypes as C
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import gym_ballenv_amd as gb  # noqa: E402
from gym_ballenv_amd import _abi  # noqa: E402

dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
N, W, K = 65536, 10, 20
env = gb.BatchedBallEnv(N, W, gb.EnvConfig(), device=dev, seed=0xBA11)
acts = env.sample_actions(K, seed=1)
env.reset()
lib = _abi.lib()


def capture():
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=torch.cuda.Stream(dev)):
        cs = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        for t in range(K):
            lib.be_step(env._ctx, C.byref(env._st), C.c_void_p(acts[t].data_ptr()), None, None, C.byref(env._out), cs)
    return g


g = capture()
for _ in range(30):
    g.replay()
torch.cuda.synchronize(dev)
print("default stream handle:", torch.cuda.current_stream(dev).cuda_stream, flush=True)


def region(stream):
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(dev)
    with torch.cuda.stream(stream):
        ev0.record(stream)
        t0 = time.perf_counter()
        g.replay()
        ev1.record(stream)
        torch.cuda.synchronize(dev)
        el = time.perf_counter() - t0
    return el * 1e6, ev0.elapsed_time(ev1) * 1e3


side = torch.cuda.Stream(dev)
hi = torch.cuda.Stream(dev, priority=-1)
for name, s in (("default", torch.cuda.current_stream(dev)), ("side", side), ("side-hiprio", hi),
                ("default", torch.cuda.current_stream(dev)), ("side", side)):
    r = [region(s) for _ in range(40)]
    print(f"{name:12s} wall {statistics.median(x for x, _ in r):7.1f} us  events {statistics.median(y for _, y in r):7.1f} us",
          flush=True)
env.close()
