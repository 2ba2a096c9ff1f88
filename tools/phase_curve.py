"""Step-kernel time against steps since reset: a fresh 65 536-env batch (W=10, defaults) is stepped
through CHUNKS x 100 graph-replayed steps (random actions), each 100-step replay timed with HIP
events, to find where the episode-phase mix (and with it the reset rate) settles.

    python tools/phase_curve.py [CHUNKS]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ctypes as C  # noqa: E402
import torch  # noqa: E402
import gym_ballenv_amd as gb  # noqa: E402
from gym_ballenv_amd import _abi  # noqa: E402

CH = int(sys.argv[1]) if len(sys.argv) > 1 else 80
N, W, T = int(os.environ.get("ENVS", 65536)), 10, 100
dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
env = gb.BatchedBallEnv(N, W, gb.EnvConfig(), device=dev, seed=0xBA11)
lib = _abi.lib()
acts = env.sample_actions(T, seed=0xBA11)
env.reset()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g, stream=torch.cuda.Stream(dev)):
    cs = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    for t in range(T):
        assert lib.be_step(env._ctx, C.byref(env._st), C.c_void_p(acts[t].data_ptr()), None, None,
                           C.byref(env._out), cs) == 0
torch.cuda.synchronize(dev)
env.reset()          # capture stepped nothing; start the curve from a fresh batch
stream = torch.cuda.current_stream(dev)
rows = []
prev = env.episode.to(torch.int64).sum().item()
for c in range(CH):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    g.replay()
    e1.record(stream)
    torch.cuda.synchronize(dev)
    eps = env.episode.to(torch.int64).sum().item()
    lens = env.ep_len.float()
    rows.append((c * T, e0.elapsed_time(e1) * 1e3 / T, (eps - prev) / T, lens.mean().item(), lens.std().item()))
    prev = eps
print("steps since reset | us/step | resets/step | ep_len mean | ep_len std")
for s, us, r, m, sd in rows:
    print(f"{s:6d}-{s + T - 1:<6d} {us:7.3f} {r:9.1f} {m:8.1f} {sd:8.1f}", flush=True)
for a, b in ((0, 1000), (1000, 2000), (2000, 4000), (4000, CH * T)):
    sel = [us for s, us, *_ in rows if a <= s < b]
    if sel:
        print(f"mean over steps [{a}, {b}): {sum(sel) / len(sel):.3f} us/step")
env.close()
