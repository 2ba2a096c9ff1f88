"""Does the freshness of the action rows change the step kernel's time?  65 536 envs, W=10, graphs
of 250 launches replayed back to back: (a) 250 action rows replayed over and over (rows stay in
the L2 / Infinity Cache), (b) a new row for every step from a 4 000-row tape (262 MB, so each row
comes from HBM), (c) like (b) but every row read once by an untimed pass just before (MALL-warm).
µs per step from HIP events over 4 000 steps, after 1 000 untimed steps."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import gym_ballenv_amd as gb  # noqa: E402
from gym_ballenv_amd import _abi  # noqa: E402

dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
N, W, CH, T = 65536, 10, 250, 4000
lib = _abi.lib()
env = gb.BatchedBallEnv(N, W, gb.EnvConfig(), device=dev, seed=0xBA11)
tape = env.sample_actions(T, seed=0xBA11)


def graphs(rows):
    gs = []
    cap = torch.cuda.Stream(dev)
    for c0 in range(0, len(rows), CH):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=cap):
            cs = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
            for t in rows[c0:c0 + CH]:
                lib.be_step(env._ctx, C.byref(env._st), C.c_void_p(tape[t].data_ptr()), None, None, C.byref(env._out), cs)
        gs.append(g)
    torch.cuda.synchronize(dev)
    return gs


def timed(gs):
    s = torch.cuda.current_stream(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(dev)
    e0.record(s)
    for g in gs:
        g.replay()
    e1.record(s)
    torch.cuda.synchronize(dev)
    return e0.elapsed_time(e1) * 1e3 / (len(gs) * CH)


env.reset()
cyc = graphs(list(range(CH)))
fresh = graphs(list(range(T)))
for _ in range(4):
    cyc[0].replay()                      # 1 000 untimed steps
torch.cuda.synchronize(dev)
big = torch.empty(512 * 1024 * 1024, dtype=torch.uint8, device=dev)   # evicts the caches
for rep in range(2):
    big.add_(1)
    a = timed([cyc[0]] * (T // CH))
    big.add_(1)
    b = timed(fresh)
    c = timed(fresh)                     # the same rows again, now read once before
    print(f"rep {rep}: cycled 250 rows {a:.3f} us/step | fresh rows {b:.3f} | same rows again {c:.3f}", flush=True)
env.close()
