"""Time be_policy_act (65536 envs, W=10, reference weights) under ablation bits.

    BALLENV_LIB=<variant .so> python tools/policy_ablate.py [dbg ...]
dbg bits (csrc/policy.hip PParams.dbg): 1 no LDS staging, 2 no MFMA, 4 no head FMAs, 8 no epilogue.
Prints one line per dbg value: mean us per launch over a graph of 200 launches.
"""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import gym_ballenv_amd as gb  # noqa: E402
from gym_ballenv_amd.policy import HipPolicy, Policy, reference_weights  # noqa: E402


def main():
    dbgs = [int(x, 0) for x in sys.argv[1:]] or [0]
    N, W, K = int(os.environ.get("ENVS", 65536)), 10, 200
    dev = torch.device("cuda:0")
    env = gb.BatchedBallEnv(N, W, gb.EnvConfig(), device=dev)
    env.reset()
    acts = env.sample_actions(50)
    for t in range(50):
        env.step(acts[t])
    pol = Policy.from_npz(reference_weights(W), W)
    for dbg in dbgs:
        os.environ["BALLENV_POLICY_DEBUG"] = str(dbg)
        hp = HipPolicy(env, pol)
        hp.act()
        s = torch.cuda.Stream(dev)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            sp = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
            for _ in range(K):
                hp._lib.be_policy_act(hp._h, C.byref(env._st), env.obs.data_ptr(), C.byref(hp._out), 7, sp)
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(3):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        print(f"{os.path.basename(os.environ.get('BALLENV_LIB', 'libballenv.so'))} dbg={dbg}: "
              f"{e0.elapsed_time(e1) / (3 * K) * 1e3:.2f} us/launch", flush=True)
        del g
        hp.close()


if __name__ == "__main__":
    main()
