"""One rank of the multi-rank engine rehearsal (tests/test_gpu_dist.py starts it under
`python -m torch.distributed.run --nproc-per-node N`, backend gloo, every rank on cuda:0).

Each rank steps its shard() of the global env batch at the defaults (13 + 5 obstacles,
TimeLimit 1000, autoreset; SURVEY.md §8(e), BASELINE config 4) with caller actions keyed by
global env id, then all_gathers the episode-statistics record with gather_stats -- the only
exchange the reference's caller has (the returns it logs).  It dumps its per-step rewards /
dones / packed obs bits, its state, its stats slots and the gathered records into --out.
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def start_lens(off, n):
    """Episode phase of global envs [off, off+n): a pure function of the global env id, so every
    split of the batch starts the same (goal changes and TimeLimit truncations inside the run)."""
    import torch
    g = torch.arange(off, off + n, dtype=torch.int64)
    return ((g * 7919) % 1000).to(torch.int32)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--envs", type=int, default=8192)
    ap.add_argument("--steps", type=int, default=120)
    ap.add_argument("--window", type=int, default=10)
    ap.add_argument("--seed", type=int, default=0xD157)
    args = ap.parse_args()

    import numpy as np
    import torch
    import torch.distributed as dist

    import gym_ballenv_amd as gb

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    off, n = gb.shard(args.envs, rank, world)
    env = gb.BatchedBallEnv(n, args.window, gb.EnvConfig(), device=dev, seed=args.seed, env_offset=off)
    env.reset()
    env.ep_len.copy_(start_lens(off, n).to(dev))
    acts = env.sample_actions(args.steps, seed=args.seed)
    T, F = args.steps, env.obs_dim
    rew = np.empty((T, n))
    done = np.empty((T, n), bool)
    obs_bits = np.empty((T, n, (F + 7) // 8), np.uint8)
    for t in range(T):
        obs, r, d, _ = env.step(acts[t])
        rew[t], done[t] = r.cpu().numpy(), d.cpu().numpy()
        obs_bits[t] = np.packbits(obs.cpu().numpy(), axis=1)
    env.status()
    per_rank = gb.gather_stats(env.stats_record())
    st = {k: v.cpu().numpy() for k, v in env.state_dict().items()}
    np.savez(os.path.join(args.out, f"rank{rank}.npz"), off=off, n=n, reward=rew, done=done, obs_bits=obs_bits,
             stats_buf=env.stats_buf.cpu().numpy(), gathered=per_rank.cpu().numpy(),
             kernel=np.array(env.kernel_name("step")), **{"state_" + k: v for k, v in st.items()})
    print(f"rank {rank}/{world}: envs [{off}, {off + n}) x {T} steps done", flush=True)
    env.close()
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
