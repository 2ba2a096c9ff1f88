"""Sibling observation formats against golden vectors made by
running the reference's own functions (tests/golden/make_golden_features.py):

* prep_state2 block counts (examples/ball_env_reinforce.py:130-172): the C oracle (CPU)
  and be_observe_blocks (GPU), bit-exact;
* the no-quadrant window of examples/potential_fields_modified.py:66-93: the oracle's
  prep_state4 window part (CPU) and BatchedBallEnv.window_only() (GPU), bit-exact.
"""
import numpy as np
import pytest
import torch

from helpers import load, window_config, window_state
from oracle import oracle


def _state(fx, key):
    st, K = window_state(fx[f"{key}_agent"], fx[f"{key}_goal"], fx[f"{key}_obst"], fx[f"{key}_nobs"])
    return st, K


def test_oracle_blocks_golden():
    fx = load("features")
    st, K = _state(fx, "blocks")
    cfg = window_config('{}', K).to_abi(st["agent"].shape[0], 5)
    np.testing.assert_array_equal(oracle.observe_blocks(cfg, st), fx["blocks_obs"])


@pytest.mark.parametrize("W", [5, 10])
def test_oracle_potential_field_window_golden(W):
    fx = load("features")
    st, K = _state(fx, f"pf{W}")
    cfg = window_config('{}', K).to_abi(st["agent"].shape[0], W)
    out = oracle.new_out(cfg)
    oracle.observe(cfg, st, out)
    np.testing.assert_array_equal(out["obs"][:, 4:], fx[f"pf{W}_obs"])


@pytest.mark.gpu
def test_gpu_blocks_golden(gpu):
    from gym_ballenv_amd import BatchedBallEnv
    fx = load("features")
    st, K = _state(fx, "blocks")
    n = st["agent"].shape[0]
    env = BatchedBallEnv(n, 5, window_config('{}', K), device=gpu)
    env.load_state_dict({k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in st.items()})
    np.testing.assert_array_equal(env.observe_blocks().cpu().numpy(), fx["blocks_obs"])
    np.testing.assert_array_equal(env.observe_blocks(f32=True).cpu().numpy(), fx["blocks_obs"].astype(np.float32))
    env.close()


@pytest.mark.gpu
@pytest.mark.parametrize("W", [5, 10])
def test_gpu_potential_field_window_golden(gpu, W):
    from gym_ballenv_amd import BatchedBallEnv
    fx = load("features")
    st, K = _state(fx, f"pf{W}")
    n = st["agent"].shape[0]
    env = BatchedBallEnv(n, W, window_config('{}', K), device=gpu)
    env.load_state_dict({k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in st.items()})
    env.observe()
    np.testing.assert_array_equal(env.window_only().cpu().numpy(), fx[f"pf{W}_obs"])
    env.close()


@pytest.mark.gpu
@pytest.mark.parametrize("ns,nd", [(13, 5), (30, 5), (0, 0), (2, 1)])
def test_gpu_blocks_vs_oracle_rollout(gpu, ns, nd):
    """Block counts of every state along a Philox rollout with autoreset (N not a multiple of 256)
    equal the oracle's on the same state: the default 13+5 obstacles (three load chunks of 6), 35
    (six chunks, the last partial), none, and 3 (one partial chunk)."""
    from gym_ballenv_amd import BatchedBallEnv, EnvConfig
    N = 3000
    env = BatchedBallEnv(N, 10, EnvConfig(time_limit=30, num_static=ns, num_dynamic=nd, obstacle_speed=[1] * nd),
                         device=gpu, seed=4)
    env.reset()
    cfg = env._abi_cfg
    for t in range(40):
        env.step()
        if t % 5 == 0:
            st = {k: getattr(env, k).cpu().numpy().copy() for k in env.STATE_KEYS}
            st["episode"] = st["episode"].view(np.uint32)
            ref = oracle.observe_blocks(cfg, st)
            np.testing.assert_array_equal(env.observe_blocks().cpu().numpy(), ref)
            np.testing.assert_array_equal(env.observe_blocks(f32=True).cpu().numpy(), ref.astype(np.float32))
    env.close()
