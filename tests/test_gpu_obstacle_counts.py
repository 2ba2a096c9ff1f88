"""GPU parity at obstacle counts past the generic kernel's register chunks.

The generic step / reset kernels (be_kernel<W, MODE, 0, 0>) hold CS = 16 static and CD = 8
dynamic obstacles per lane group in registers; further obstacles go through the overflow loops
(`kb >= CS` / `kb >= CD`), and dynamic obstacle k draws field k % 5 of Philox block k / 5, so
more than 5 (10, 15) dynamic obstacles need a second (third, fourth) block.  The BASELINE configs
never reach these paths (13 + 5); these cases run them -- up to be_config_check's maxima (64
static; 16 dynamic, as each dynamic obstacle starts on its own goal and there are at most 16
goals) -- bit-exact against the
oracle (ballenv_env.py:113-167 reset, :232-289 step, :323-353 move_obstacles), with autoreset,
the TimeLimit, terminal obs, masked resets and the stats.
"""
import numpy as np
import pytest
import torch

from oracle import oracle
from test_gpu_parity import assert_state_equal, make_env

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("ns,nd,W,N,given", [
    (40, 12, 10, 3000, False),    # both overflow loops, three Philox blocks for the dynamics
    (64, 16, 7, 1000, True),      # be_config_check's maxima, four Philox blocks, caller actions
    (0, 9, 18, 500, False),       # no statics, runtime-W kernel (W = 18 has no compiled instance)
    (20, 0, 10, 2000, True),      # no dynamics
    (17, 6, 5, 4096, True),       # one past each chunk / block boundary
])
def test_generic_kernel_obstacle_counts_vs_oracle(gpu, ns, nd, W, N, given):
    from gym_ballenv_amd.config import EnvConfig
    speeds = [1 + (k % 3) for k in range(nd)]
    goals = [((37 * g + 12) % 500, (53 * g + 122) % 500) for g in range(max(5, nd))]   # pairwise distinct
    cfg_py = EnvConfig(num_static=ns, num_dynamic=nd, obstacle_speed=speeds, goals=goals, time_limit=25,
                       goal_change_step=4, autoreset=True)
    cfg = cfg_py.to_abi(N, W, seed=31)
    env = make_env(cfg_py, N, W, gpu, seed=31, terminal_obs=True)
    assert env.kernel_name("step").endswith(", 0, 0, false>"), env.kernel_name("step")   # the generic kernel
    st = oracle.new_state(cfg)
    out = oracle.new_out(cfg, terminal=True)
    oracle.reset(cfg, st, out)
    np.testing.assert_array_equal(env.reset().cpu().numpy(), out["obs"])
    assert_state_equal(env, st, "reset")
    acts = env.sample_actions(40, seed=8) if given else None
    rng = np.random.default_rng(ns * 100 + nd)
    n_done = 0
    for t in range(40):
        if t == 20:   # a masked reset mid-run (the block-cooperative reset path with many obstacles)
            mask = (rng.random(N) < 0.3).astype(np.uint8)
            oracle.reset(cfg, st, out, mask=mask)
            np.testing.assert_array_equal(env.reset(torch.from_numpy(mask)).cpu().numpy(), out["obs"], err_msg="masked reset")
            assert_state_equal(env, st, "masked reset")
        out["terminal_obs"][:] = 0
        env.terminal_obs.zero_()
        if given:
            oracle.step(cfg, st, out, actions=acts[t].cpu().numpy())
            obs, reward, done, info = env.step(acts[t])
        else:
            oracle.step(cfg, st, out)
            obs, reward, done, info = env.step()
        d = done.cpu().numpy()
        n_done += int(d.sum())
        np.testing.assert_array_equal(reward.cpu().numpy(), out["reward"], err_msg=f"reward t={t}")
        np.testing.assert_array_equal(d, out["done"].astype(bool), err_msg=f"done t={t}")
        np.testing.assert_array_equal(info["truncated"].cpu().numpy(), out["truncated"].astype(bool), err_msg=f"t={t}")
        np.testing.assert_array_equal(obs.cpu().numpy(), out["obs"], err_msg=f"obs t={t}")
        np.testing.assert_array_equal(info["final_return"].cpu().numpy()[d], out["final_return"][d])
        np.testing.assert_array_equal(info["final_len"].cpu().numpy()[d], out["final_len"][d])
        np.testing.assert_array_equal(info["terminal_obs"].cpu().numpy(), out["terminal_obs"], err_msg=f"terminal t={t}")
        assert_state_equal(env, st, f"t={t}")
    assert n_done > 0
    s_gpu = env.stats_record().cpu().numpy()
    s_orc = out["stats"]
    assert s_gpu[0] == s_orc[0] and s_gpu[3] == s_orc[3] and s_gpu[4] == s_orc[4] and s_gpu[5] == s_orc[5]
    np.testing.assert_allclose(s_gpu[1:3], s_orc[1:3], rtol=1e-12, atol=1e-9)
    env.status()
    env.close()
