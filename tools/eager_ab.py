"""Host cost of BatchedBallEnv.step() per call: the current class against an earlier one,
interleaved, the bench's eager_step method (65 536 envs, W=10, actions from acts.random_ each step,
1000 calls).  The baseline class file is argv[1] (default tools/diag/batched_r04.py = `git show
3673bc0:gym-ballenv_amd/batched.py`; round 6: tools/eager_base/batched_head.py = the class before the
raw-stream call), its label argv[2].
"""
import importlib.util
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import gym_ballenv_amd as gb  # noqa: E402

BASE = sys.argv[1] if len(sys.argv) > 1 else "tools/diag/batched_r04.py"
LABEL = sys.argv[2] if len(sys.argv) > 2 else "r04"
spec = importlib.util.spec_from_file_location("gym_ballenv_amd.batched_base", os.path.join(ROOT, BASE))
old = importlib.util.module_from_spec(spec)
spec.loader.exec_module(old)


def run(cls, T=1000, N=65536):
    env = cls(N, 10, gb.EnvConfig(), device="cuda:0", seed=0xBA11)
    env.reset()
    acts = torch.empty(N, dtype=torch.uint8, device="cuda:0")
    for _ in range(200):
        acts.random_(0, 9)
        env.step(acts)
    torch.cuda.synchronize()
    call = 0.0
    pc = time.perf_counter
    t0 = pc()
    for _ in range(T):
        acts.random_(0, 9)
        c0 = pc()
        env.step(acts)
        call += pc() - c0
    torch.cuda.synchronize()
    el = pc() - t0
    env.status()
    env.close()
    return call / T * 1e6, el / T * 1e6


for rep in range(int(os.environ.get("REPS", "3"))):
    for name, cls in ((LABEL, old.BatchedBallEnv), ("new", gb.BatchedBallEnv)):
        c, it = run(cls)
        print(f"{name} rep {rep}: host us per step() call {c:.2f}, wall us per loop iteration {it:.2f}", flush=True)
