"""Time be_board_step (createBoard profile, 65536 envs, 6 statics, random actionArray moves)
with and without the feature pass and autoreset: where the step's time goes.

    python tools/board_ablate.py
"""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import gym_ballenv_amd as gb  # noqa: E402


def run(N, T, features, autoreset, time_limit=1000):
    dev = torch.device("cuda:0")
    b = gb.BatchedBoard(N, 6, device=dev, seed=0xB0A2D, autoreset=autoreset, time_limit=time_limit)
    b.reset()
    acts = torch.randint(0, 4, (T, N), dtype=torch.uint8, device=dev)
    out = b._out
    if not features:
        out = type(out)(None, *[getattr(out, f[0]) for f in out._fields_[1:]])
    lib = b._lib
    g = torch.cuda.CUDAGraph()
    cap = torch.cuda.Stream(dev)
    with torch.cuda.graph(g, stream=cap):
        sp = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        for t in range(T):
            lib.be_board_step(b._h, C.byref(b._st), C.c_void_p(acts[t].data_ptr()), None, C.byref(out), sp)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    dones = int(b.done.sum())
    b.status()
    b.close()
    return e0.elapsed_time(e1) / T * 1e3, dones


if __name__ == "__main__":
    N, T = 65536, 200
    for feats, ar in ((True, True), (False, True), (True, False), (False, False)):
        us, d = run(N, T, feats, ar)
        print(f"features={feats} autoreset={ar}: {us:.2f} us/step (dones in last step {d})", flush=True)
