"""Single-env BallEnv with the reference's gym.Env surface, on the GPU engine.

Drop-in for ``gym.make('gymball-v0')`` (gym_ballenv/__init__.py:4-11) as used by
examples/ball_cnn_ac3.py: ``reset()`` / ``step((dx, dy))`` return the
reference's state array ``[(ax, ay), (gx, gy), dist, (ox, oy)...]``
(ballenv_env.py:127,147,163,271-274), ``env.unwrapped`` exposes the attributes
the driver reads (ballenv_env.py:49-66; ball_cnn_ac3.py:390-393,404,612) and the
window observation comes from the GPU kernel: replace ``prep_state4(state, W)``
(ball_cnn_ac3.py:384-412) with ``env.unwrapped.window_obs(W)``.

This is a thin wrapper around a 1-env :class:`BatchedBallEnv` (autoreset off,
like the reference, where stepping after ``done`` is allowed) -- every physics
and observation computation runs in the HIP kernels.
"""
from __future__ import annotations

import math
from typing import Optional

import numpy as np
import torch

from .batched import BatchedBallEnv
from .config import EnvConfig
from .spaces import Box, Discrete

ENV_ID = "gymball-v0"


class BallEnv:
    metadata = {"render.modes": ["human", "rgb_array"], "video.frames_per_second": 100}

    def __init__(self, window: int = 5, config: Optional[EnvConfig] = None, device="cuda",
                 seed: Optional[int] = None, time_limit: int = 0):
        cfg = config if config is not None else EnvConfig()
        cfg.autoreset = False
        cfg.time_limit = int(time_limit)
        self._window = int(window)
        self._device = torch.device(device)
        self._seed = int(seed) if seed is not None else int(np.random.randint(0, 2**31 - 1))
        self._make(cfg)
        self.viewer = None

    def _make(self, cfg: EnvConfig):
        self._env = BatchedBallEnv(1, self._window, cfg, device=self._device, seed=self._seed)
        self.state = None
        self._done_steps = 0

    # ---- reference attribute names (ballenv_env.py:49-66)
    @property
    def radius_rand_person(self):
        return self._env.cfg.radius_obstacle

    @property
    def radius_ctrl_person(self):
        return self._env.cfg.radius_agent

    @property
    def speedx_ctrl_person(self):
        return self._env.cfg.speed_x

    @property
    def speedy_ctrl_person(self):
        return self._env.cfg.speed_y

    @property
    def threshold_goal(self):
        return self._env.cfg.threshold_goal

    @property
    def total_reward_accumulated(self) -> float:
        return float(self._env.ep_return[0])

    @property
    def unwrapped(self):
        return self

    @property
    def action_space(self) -> Discrete:
        return Discrete(len(self._env.cfg.actions))

    @property
    def observation_space(self) -> Box:
        return self._env.observation_space

    @property
    def batched(self) -> BatchedBallEnv:
        return self._env

    # ---- gym.Env protocol
    def customize_environment(self, args) -> None:
        cfg = EnvConfig.from_args(args, self._env.cfg)
        self._env.close()
        self._make(cfg)

    def seed(self, seed=None):
        self._seed = int(seed) if seed is not None else int(np.random.randint(0, 2**31 - 1))
        cfg = self._env.cfg
        self._env.close()
        self._make(cfg)
        return [self._seed]

    def reset(self):
        self._env.reset()
        self.state = self._host_state()
        return self.state

    def step(self, action):
        """action: (dx, dy) as BallEnv.step takes it, or an index into the action table."""
        if isinstance(action, (tuple, list, np.ndarray)) and len(action) == 2:
            d = torch.tensor([[int(action[0]), int(action[1])]], dtype=torch.int16, device=self._device)
            _, reward, done, info = self._env.step(deltas=d)
        else:
            a = torch.tensor([int(action)], dtype=torch.uint8, device=self._device)
            _, reward, done, info = self._env.step(actions=a)
        self.state = self._host_state()
        r, dn = float(reward[0]), bool(done[0])
        return self.state, r, dn, {"truncated": bool(info["truncated"][0])}

    def window_obs(self, window: Optional[int] = None) -> torch.Tensor:
        """(1, 4+W^2) float32 on the device: what prep_state4(state, W) returns."""
        if window is not None and window != self._window:
            raise ValueError(f"this env was built for window={self._window}")
        return self._env.obs.float()

    def check_overlap(self, tup1, tup2) -> bool:
        """ballenv_env.py:185-191 (host helper kept for API compatibility)."""
        d = math.sqrt(math.pow(tup1[0] - tup2[0], 2) + math.pow(tup1[1] - tup2[1], 2))
        return not d > (self.radius_rand_person + self.radius_ctrl_person)

    def calculate_distance(self, tup1, tup2) -> float:
        return math.sqrt(math.pow(tup1[0] - tup2[0], 2) + math.pow(tup1[1] - tup2[1], 2))

    def render(self, mode: str = "rgb_array", close: bool = False):
        from .render import render_env0
        return render_env0(self._env, mode=mode)

    def close(self):
        self._env.close()

    # ---- helpers
    def _host_state(self):
        e = self._env
        ag = e.agent[0].tolist()
        go = e.goal[0].tolist()
        st = [tuple(p) for p in e.static_obs[:e.cfg.num_static, 0].tolist()]
        dy = [tuple(p) for p in e.dyn_obs[:e.cfg.num_dynamic, 0].tolist()]
        self.goal_x, self.goal_y = go
        state = [tuple(ag), tuple(go), float(e.prev_dist[0])] + st + dy
        return np.array(state, dtype=object)


class TimeLimit:
    """gym 0.10.9 TimeLimit semantics for gym.make (max_episode_steps=1000)."""

    def __init__(self, env: BallEnv, max_episode_steps: int = 1000):
        self.env = env
        self._max_episode_steps = max_episode_steps
        self._elapsed_steps = 0

    def reset(self):
        self._elapsed_steps = 0
        return self.env.reset()

    def step(self, action):
        obs, reward, done, info = self.env.step(action)
        self._elapsed_steps += 1
        if self._elapsed_steps >= self._max_episode_steps:
            done = True
        return obs, reward, done, info

    def __getattr__(self, name):
        return getattr(self.env, name)

    @property
    def unwrapped(self):
        return self.env


def make(env_id: str = ENV_ID, **kwargs):
    """gym.make('gymball-v0') equivalent: BallEnv under a 1000-step TimeLimit."""
    if env_id != ENV_ID:
        raise ValueError(f"unknown env id {env_id!r} (only {ENV_ID!r})")
    return TimeLimit(BallEnv(**kwargs), max_episode_steps=1000)
