"""gym_ballenv_amd -- MI355X-native batched BallEnv step engine.

Drop-in for the hot path of ranok92/gym-ballenv: BallEnv.step/reset
(gym_ballenv/envs/ballenv_env.py) + the prep_state4 W x W window observation
(examples/ball_cnn_ac3.py), as hand-written gfx950 HIP kernels behind the C ABI
of include/ballenv.h (libballenv.so, built in-tree).

    import gym_ballenv_amd as gb
    env = gb.BatchedBallEnv(65536, window=10)          # (N,) struct-of-arrays on the GPU
    obs = env.reset()
    obs, reward, done, info = env.step(actions)         # one kernel launch

    env = gb.make('gymball-v0', window=5)               # single-env gym surface
"""
from .config import EnvConfig, MOVE_LIST, step_bytes, survey_step_bytes
from .spaces import Box, Discrete
from ._abi import BallEnvError


def __getattr__(name):
    # torch-dependent parts load lazily so the config / ABI helpers import fast
    if name == "BatchedBallEnv":
        from .batched import BatchedBallEnv
        return BatchedBallEnv
    if name in ("BallEnv", "make", "TimeLimit", "ENV_ID"):
        from . import envs
        return getattr(envs, name)
    if name in ("Policy", "HipPolicy", "torch_select_action"):
        from . import policy
        return getattr(policy, name)
    if name in ("Rollout", "a2c_losses", "a2c_update"):
        from . import rollout
        return getattr(rollout, name)
    if name == "BatchedBoard":
        from .board import BatchedBoard
        return BatchedBoard
    if name in ("shard", "gather_stats", "combine_stats"):
        from . import distributed
        return getattr(distributed, name)
    raise AttributeError(name)


__all__ = ["EnvConfig", "MOVE_LIST", "step_bytes", "survey_step_bytes", "Box", "Discrete", "BallEnvError", "BatchedBallEnv",
           "BallEnv", "make", "TimeLimit", "shard", "gather_stats", "combine_stats", "Policy", "HipPolicy",
           "torch_select_action", "Rollout", "a2c_losses", "a2c_update", "BatchedBoard"]
