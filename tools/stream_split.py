"""Does splitting the env batch over S concurrent streams (independent env shards,
one be_step chain per stream, fork/join inside one captured graph) raise
throughput of the latency-bound step kernel?

    python tools/stream_split.py [N] [S ...]      (default 65536; S = 1 2 4)
Also times the config-5 pair (be_policy_act + be_step) per stream.
"""
import ctypes as C
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import gym_ballenv_amd as gb  # noqa: E402
from gym_ballenv_amd.policy import HipPolicy, Policy, reference_weights  # noqa: E402


def run(N, S, K, with_policy):
    dev = torch.device("cuda:0")
    n = N // S
    envs = [gb.BatchedBallEnv(n, 10, gb.EnvConfig(), device=dev, seed=0xBA11, env_offset=i * n) for i in range(S)]
    for e in envs:
        e.reset()
    acts = [e.sample_actions(K) for e in envs]
    pols = None
    if with_policy:
        pol = Policy.from_npz(reference_weights(10), 10)
        pols = [HipPolicy(e, pol) for e in envs]
    torch.cuda.synchronize()
    lib = envs[0]._lib
    streams = [torch.cuda.Stream(dev) for _ in range(S)]
    cap = torch.cuda.Stream(dev)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=cap):
        for s in streams:
            s.wait_stream(cap)
        for t in range(K):
            for i, (e, s) in enumerate(zip(envs, streams)):
                sp = C.c_void_p(s.cuda_stream)
                if with_policy:
                    hp = pols[i]
                    lib.be_policy_act(hp._h, C.byref(e._st), e.obs.data_ptr(), C.byref(hp._out), 7, sp)
                    a = hp.action.data_ptr()
                else:
                    a = acts[i][t].data_ptr()
                lib.be_step(e._ctx, C.byref(e._st), C.c_void_p(a), None, None, C.byref(e._out), sp)
        for s in streams:
            cap.wait_stream(s)
    g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / 3
    for e in envs:
        e.status()
    print(f"N={N} S={S} policy={with_policy}: {el / K * 1e6:.2f} us/step  {N * K / el:.3e} env-steps/s", flush=True)
    del g
    if pols:
        for p in pols:
            p.close()
    for e in envs:
        e.close()


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    Ss = [int(x) for x in sys.argv[2:]] or [1, 2, 4]
    for wp in (False, True):
        for S in Ss:
            run(N, S, 200, wp)


if __name__ == "__main__":
    main()
