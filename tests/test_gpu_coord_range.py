"""GPU: the int16 coordinate range of the dynamic obstacles, and the caller's current device.

The reference's dynamic obstacles are unbounded Python ints with no clamp
(gym_ballenv/envs/ballenv_env.py:334-347); the engine stores them as int16.  A config whose
episodes are bounded (autoreset + time limit) cannot leave int16 -- be_config_check rejects the
rest of those (tests/test_abi_host.py) -- but with time_limit 0 or autoreset 0 an obstacle can
walk out.  Then every step kernel raises BE_STATUS_COORD_RANGE, which status() turns into
BallEnvError, and stores the coordinate wrapped to two's complement int16.  These tests park
obstacles on the int16 edge and drive them across it: in tape (parity) mode through the generic
kernel, and in Philox mode through each fixed-shape kernel, bit-exact against the oracle (which
wraps and flags the same way).
"""
import numpy as np
import pytest
import torch

from oracle import oracle
from test_gpu_episode import fixed_step_kernel
from test_gpu_parity import KEYS, load_np_state, make_env, np_state

pytestmark = pytest.mark.gpu

MSG = "int16 coordinate range"


def _assert_state(env, st, a, k, msg):
    got = np_state(env)
    for key in KEYS:
        g = got[key][:, a:a + k] if key in ("static_obs", "dyn_obs", "dyn_goal") else got[key][a:a + k]
        np.testing.assert_array_equal(g, st[key], err_msg=f"{msg}: state[{key}]")


def test_coord_range_tape_mode(gpu):
    """Tape (parity) mode, generic kernel: three obstacles parked on the int16 edge take the
    reference's random move (u = 99 >= rd_th_obs, then OBS_MOVES[m], ballenv_env.py:339-347)
    across it -- +x from 32767, +y from 32767, -x from -32768 -- and wrap."""
    from gym_ballenv_amd import _abi
    from gym_ballenv_amd.config import EnvConfig
    cfg_py = EnvConfig(autoreset=False, time_limit=0)
    N, W = 64, 10
    cfg = cfg_py.to_abi(N, W, seed=5)
    st = oracle.new_state(cfg)
    out = oracle.new_out(cfg)
    assert oracle.reset(cfg, st, out) == 0
    env = make_env(cfg_py, N, W, gpu, seed=5)
    env.reset()
    edge = st["dyn_obs"].copy()
    edge[0, :, 0] = 32767                 # goal (12, 122):  move (1, 0)  -> x 32768
    edge[1, :] = (200, 32767)             # goal (123, 93):  move (1, 1)  -> y 32768
    edge[2, :] = (-32768, 300)            # goal (87, 150):  move (-1,-1) -> x -32769
    st["dyn_obs"][:] = edge
    load_np_state(env, st)
    tape = np.zeros((5, 2, N), np.int16)  # obstacles 3, 4: u = 0 < 60, the directed move
    tape[0:3, 0] = 99
    tape[0, 1], tape[1, 1], tape[2, 1] = 2, 0, 7
    acts = np.full(N, 5, np.uint8)        # the agent stays
    status = oracle.step(cfg, st, out, actions=acts, tape=tape)
    assert status & 8, status
    obs, reward, done, _ = env.step(torch.from_numpy(acts).to(gpu), draw_tape=torch.from_numpy(tape).to(gpu))
    with pytest.raises(_abi.BallEnvError, match=MSG):
        env.status()
    env.status()                          # read-and-clear: the next poll is clean
    got = np_state(env)
    np.testing.assert_array_equal(got["dyn_obs"][0, :, 0], np.full(N, -32768, np.int16))
    np.testing.assert_array_equal(got["dyn_obs"][1, :, 1], np.full(N, -32768, np.int16))
    np.testing.assert_array_equal(got["dyn_obs"][2, :, 0], np.full(N, 32767, np.int16))
    np.testing.assert_array_equal(got["dyn_obs"][1, :, 0], np.full(N, 201, np.int16))
    np.testing.assert_array_equal(got["dyn_obs"][2, :, 1], np.full(N, 299, np.int16))
    _assert_state(env, st, 0, N, "after the wrap")
    np.testing.assert_array_equal(reward.cpu().numpy(), out["reward"])
    np.testing.assert_array_equal(done.cpu().numpy(), out["done"].astype(bool))
    np.testing.assert_array_equal(obs.cpu().numpy(), out["obs"])
    env.close()


@pytest.mark.parametrize("W,N,a", [(10, 32768, 20000), (5, 4096, 1024), (10, 131072, 100000)])
def test_coord_range_fixed_kernels(gpu, W, N, a):
    """Philox mode, the fixed-shape kernels (step2_kernel, stepw_kernel, the one-lane kernel) at
    time_limit 0: obstacle 0 parked at x = 32767 and obstacle 3 at y = -32768 in every env; the
    envs whose draw is a random move across the edge wrap, the kernel flags the status word, and
    three steps match the oracle bit for bit on a 2048-env slice (global ids a .. a+2047)."""
    from gym_ballenv_amd import _abi
    from gym_ballenv_amd.config import EnvConfig
    cfg_py = EnvConfig(time_limit=0)
    k = 2048
    env = make_env(cfg_py, N, W, gpu, seed=0xBA11)
    assert env.kernel_name("step") == fixed_step_kernel(W, N)
    cfg = cfg_py.to_abi(k, W, env_offset=a, seed=0xBA11)
    st = oracle.new_state(cfg)
    out = oracle.new_out(cfg)
    oracle.reset(cfg, st, out)
    env.reset()
    full = np_state(env)
    full["dyn_obs"][0, :, 0] = 32767
    full["dyn_obs"][3, :, 1] = -32768
    load_np_state(env, full)
    st["dyn_obs"][0, :, 0] = 32767
    st["dyn_obs"][3, :, 1] = -32768
    _assert_state(env, st, a, k, "parked")
    acts = env.sample_actions(3, seed=77)
    wrapped = 0
    for t in range(3):
        status = oracle.step(cfg, st, out, actions=acts[t, a:a + k].cpu().numpy())
        obs, reward, done, _ = env.step(acts[t])
        if t == 0:
            assert status & 8, status
            d = np_state(env)["dyn_obs"]
            wrapped = int((d[0, :, 0] == -32768).sum() + (d[3, :, 1] == 32767).sum())
        if status & 8:                    # obstacles still on the edge may cross on a later step
            with pytest.raises(_abi.BallEnvError, match=MSG):
                env.status()
        else:
            env.status()
        sl = slice(a, a + k)
        np.testing.assert_array_equal(reward[sl].cpu().numpy(), out["reward"], err_msg=f"reward t={t}")
        np.testing.assert_array_equal(done[sl].cpu().numpy(), out["done"].astype(bool), err_msg=f"done t={t}")
        np.testing.assert_array_equal(obs[sl].cpu().numpy(), out["obs"], err_msg=f"obs t={t}")
        _assert_state(env, st, a, k, f"t={t}")
    # ~13 % of obstacle 0 (3 of 9 random moves go +x) and ~18 % of obstacle 3 wrap
    assert N * 0.05 < wrapped < N * 0.5, wrapped
    env.close()


def test_entry_points_keep_the_callers_device(gpu):
    """Every entry point makes the context's device current for the call and restores the
    caller's current device (include/ballenv.h): torch's current device is unchanged across
    reset / step / rollout / observe / sample_actions / status / save/load / the policy.  With
    two or more GPUs the env lives on the last one while the caller's current device is 0."""
    from gym_ballenv_amd import BatchedBallEnv
    from gym_ballenv_amd.config import EnvConfig
    from gym_ballenv_amd.policy import HipPolicy, Policy
    ndev = torch.cuda.device_count()
    if ndev < 2:   # env and caller on the same device: DeviceGuard would switch nothing
        pytest.skip("needs two GPUs: with one, the caller's device is the context's and nothing is restored")
    dev = torch.device("cuda", ndev - 1)
    torch.cuda.set_device(0)
    env = BatchedBallEnv(4096, 10, EnvConfig(), device=dev)
    assert torch.cuda.current_device() == 0
    acts = env.sample_actions(4)
    assert torch.cuda.current_device() == 0
    env.reset()
    assert torch.cuda.current_device() == 0
    env.step(acts[0])
    env.step()
    assert torch.cuda.current_device() == 0
    env.rollout(acts[1:3])
    env.observe()
    env.observe_blocks()
    blob = env.save_state()
    env.load_state(blob)
    env.status()
    assert torch.cuda.current_device() == 0
    torch.manual_seed(0)
    hp = HipPolicy(env, Policy(10).to(dev))
    hp.act(env.obs)
    assert torch.cuda.current_device() == 0
    hp.close()
    env.close()
    assert torch.cuda.current_device() == 0
