"""Multi-rank engine rehearsal on one GPU (BASELINE config 4's code path).

A fresh child `python -m torch.distributed.run --nproc-per-node {2, 8}` (gloo; every rank on
cuda:0; started as a new process, never an exec) runs tests/dist_engine_worker.py: each rank
steps its shard() of the global batch (8 192, or config 4's 262 144) for 120 / 40 default-config steps (episode phases set from the global
env id, so goal changes and TimeLimit truncations happen) and all_gathers its stats record.
This process then runs the whole batch on one rank and checks, bit for bit, that the ranks'
per-env rewards / dones / obs, their final states, their per-wave stats slots and the gathered
records equal the matching rows of the one-rank run (Philox streams are keyed by global env id),
and that the last rank's last 1 024 envs equal the oracle run on the same global ids.
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("E,T,world", [(8192, 120, 2), (262144, 40, 8)], ids=["2x4096", "config4_8x32768"])
def test_multi_rank_engine_matches_one_rank(gpu, tmp_path, E, T, world):
    """2 ranks x 4 096 envs for 120 steps, and BASELINE config 4's split (262 144 envs over 8
    ranks of 32 768) for 40 steps.  At config 4 the ranks step on step2_kernel and the one-rank
    run of the whole batch on the one-lane kernel (the batch-size dispatch), so the check is
    also a cross-kernel one."""
    import gym_ballenv_amd as gb
    from dist_engine_worker import start_lens
    W, seed = 10, 0xD157
    env_vars = dict(os.environ, MASTER_ADDR="127.0.0.1", PYTHONPATH=ROOT, OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
           os.path.join(HERE, "dist_engine_worker.py"), "--out", str(tmp_path), "--envs", str(E),
           "--steps", str(T), "--window", str(W), "--seed", str(seed)]
    r = subprocess.run(cmd, cwd=ROOT, env=env_vars, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    ranks = [dict(np.load(tmp_path / f"rank{i}.npz")) for i in range(world)]

    # the same global batch on one rank
    env = gb.BatchedBallEnv(E, W, gb.EnvConfig(), device=gpu, seed=seed)
    env.reset()
    env.ep_len.copy_(start_lens(0, E).to(gpu))
    acts = env.sample_actions(T, seed=seed)
    rew = np.empty((T, E))
    done = np.empty((T, E), bool)
    bits = np.empty((T, E, (env.obs_dim + 7) // 8), np.uint8)
    for t in range(T):
        obs, rw, d, _ = env.step(acts[t])
        rew[t], done[t], bits[t] = rw.cpu().numpy(), d.cpu().numpy(), np.packbits(obs.cpu().numpy(), axis=1)
    env.status()
    st = {k: v.cpu().numpy() for k, v in env.state_dict().items()}
    slots = env.stats_buf.cpu().numpy()
    assert env.kernel_name("step") == ("step2_kernel<10, 13, 5, true>" if E <= 98304 else "be_kernel<10, 0, 13, 5, false>")   # (262 144: past the one-lane pool bound)

    assert done.sum() > E * T // 2000, "episodes must finish and autoreset during the run"
    for i, rk in enumerate(ranks):
        off, n = int(rk["off"]), int(rk["n"])
        assert (off, n) == gb.shard(E, i, world)
        assert str(rk["kernel"]) == "step2_kernel<10, 13, 5, true>"
        sl = slice(off, off + n)
        np.testing.assert_array_equal(rk["reward"], rew[:, sl], err_msg=f"rank {i} reward")
        np.testing.assert_array_equal(rk["done"], done[:, sl], err_msg=f"rank {i} done")
        np.testing.assert_array_equal(rk["obs_bits"], bits[:, sl], err_msg=f"rank {i} obs")
        for k, v in st.items():
            want = v[:, sl] if k in ("static_obs", "dyn_obs", "dyn_goal") else v[sl]
            np.testing.assert_array_equal(rk["state_" + k], want, err_msg=f"rank {i} state[{k}]")
        # stats slots (one per 32 envs): a rank's slots are the one-rank run's slots of its env range
        se = E // slots.shape[0]
        assert se == 32 and off % se == 0 and n % se == 0
        np.testing.assert_array_equal(rk["stats_buf"], slots[off // se:(off + n) // se], err_msg=f"rank {i} stats")
    # every rank gathered the same (world, 8) records: each rank's own reduction of its slots
    for rk in ranks:
        np.testing.assert_array_equal(rk["gathered"], ranks[0]["gathered"])
    g = ranks[0]["gathered"]
    for i, rk in enumerate(ranks):
        b = torch.from_numpy(rk["stats_buf"])
        rec = b.sum(0)
        rec[4], rec[5] = b[:, 4].min(), b[:, 5].max()
        r = rec.numpy()   # (the rank reduced on the GPU: sums in its own order)
        np.testing.assert_array_equal(g[i][[0, 4, 5]], r[[0, 4, 5]])
        np.testing.assert_allclose(g[i][1:4], r[1:4], rtol=1e-12)
    comb = gb.combine_stats(torch.from_numpy(g))
    one = env.episode_stats()
    assert comb["episodes"] == one["episodes"] and comb["min_return"] == one["min_return"]
    assert comb["max_return"] == one["max_return"]
    assert comb["mean_length"] == pytest.approx(one["mean_length"], rel=1e-12)
    assert comb["mean_return"] == pytest.approx(one["mean_return"], rel=1e-12)

    # not only a self-comparison: the last rank's last 1 024 envs against the oracle, step by step
    from oracle import oracle
    rk = ranks[-1]
    off, n = int(rk["off"]), int(rk["n"])
    k = 1024
    a = off + n - k
    cfg = gb.EnvConfig().to_abi(k, W, env_offset=a, seed=seed)
    ost = oracle.new_state(cfg)
    oout = oracle.new_out(cfg)
    oracle.reset(cfg, ost, oout)
    ost["ep_len"][:] = start_lens(a, k).numpy()
    loc = slice(a - off, a - off + k)
    for t in range(T):
        oracle.step(cfg, ost, oout, actions=acts[t, a:a + k].cpu().numpy())
        np.testing.assert_array_equal(rk["reward"][t, loc], oout["reward"], err_msg=f"oracle reward t={t}")
        np.testing.assert_array_equal(rk["done"][t, loc], oout["done"].astype(bool), err_msg=f"oracle done t={t}")
        np.testing.assert_array_equal(rk["obs_bits"][t, loc], np.packbits(oout["obs"], axis=1), err_msg=f"oracle obs t={t}")
    for key in ("agent", "goal", "ep_len", "static_obs", "dyn_obs", "dyn_goal"):
        got = rk["state_" + key]
        got = got[:, loc] if key in ("static_obs", "dyn_obs", "dyn_goal") else got[loc]
        np.testing.assert_array_equal(got, ost[key], err_msg=f"oracle state[{key}]")
    env.close()
