"""Shared test helpers: golden fixtures -> configs / SoA states / tapes."""
from __future__ import annotations

import json
import os
from types import SimpleNamespace

import numpy as np

from gym_ballenv_amd.config import EnvConfig

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

ENV_MAP = {"radius_rand_person": "radius_obstacle", "radius_ctrl_person": "radius_agent",
           "speedx_ctrl_person": "speed_x", "speedy_ctrl_person": "speed_y", "threshold_goal": "threshold_goal"}
STRIP_MAP = {"_stripobsx": "strip_obs_x", "_stripobsy": "strip_obs_y", "_stripgoalx": "strip_goal_x",
             "_stripgoaly": "strip_goal_y", "_stripagentx": "strip_agent_x", "_stripagenty": "strip_agent_y"}


def load(name):
    return dict(np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False))


def env_config(cfg_json, autoreset=False, time_limit=0) -> EnvConfig:
    d = json.loads(str(cfg_json))
    env = d.pop("env", {}) or {}
    strips = d.pop("strips", {}) or {}
    d.pop("window", None)
    c = EnvConfig.from_args(SimpleNamespace(**d))
    for k, v in env.items():
        setattr(c, ENV_MAP[k], v)
    for k, v in strips.items():
        setattr(c, STRIP_MAP[k], v)
    c.autoreset = autoreset
    c.time_limit = time_limit
    return c


def window_config(env_json, nobs) -> EnvConfig:
    c = EnvConfig(num_static=nobs, num_dynamic=0, obstacle_speed=[], goals=[], autoreset=False, time_limit=0)
    for k, v in json.loads(str(env_json)).items():
        setattr(c, ENV_MAP[k], v)
    return c


def init_state(fx, prefix="init_"):
    """SoA numpy state (BatchedBallEnv layout) from a fixture's init_* arrays."""
    E = fx[prefix + "agent"].shape[0]
    st = dict(agent=fx[prefix + "agent"].astype(np.int16).copy(), goal=fx[prefix + "goal"].astype(np.int16).copy(),
              prev_dist=fx[prefix + "prev_dist"].astype(np.float64).copy(),
              total_dist=fx[prefix + "total_dist"].astype(np.float64).copy(), ep_return=np.zeros(E),
              ep_len=(fx[prefix + "ep_len"].astype(np.int32).copy() if prefix + "ep_len" in fx
                      else np.zeros(E, np.int32)), episode=np.ones(E, np.uint32))
    s = fx[prefix + "static"]
    d = fx[prefix + "dyn"]
    st["static_obs"] = np.ascontiguousarray(s.transpose(1, 0, 2).astype(np.int16)) if s.shape[1] else np.zeros((1, E, 2), np.int16)
    st["dyn_obs"] = np.ascontiguousarray(d.transpose(1, 0, 2).astype(np.int16)) if d.shape[1] else np.zeros((1, E, 2), np.int16)
    g = fx[prefix + "dyn_goal"]
    st["dyn_goal"] = np.ascontiguousarray(g.T.astype(np.uint8)) if g.shape[1] else np.zeros((1, E), np.uint8)
    return st


def step_tape(fx, t):
    """(Nd, 2, E) int16 draw tape of step t from a rollout fixture's (E, T, Nd, 2) tape."""
    return np.ascontiguousarray(fx["tape"][:, t].transpose(1, 2, 0).astype(np.int16))


def window_state(agent, goal, obst, nobs, far=-20000):
    """SoA state for a windows fixture: obstacles padded with far-away parking spots."""
    n, K = obst.shape[0], max(int(nobs.max()), 1)
    so = np.full((K, n, 2), far, np.int16)
    for i in range(n):
        k = int(nobs[i])
        if k:
            so[:k, i] = obst[i, :k]
    return dict(agent=agent.astype(np.int16).copy(), goal=goal.astype(np.int16).copy(), prev_dist=np.zeros(n),
                total_dist=np.ones(n), ep_return=np.zeros(n), ep_len=np.zeros(n, np.int32),
                episode=np.zeros(n, np.uint32),
                static_obs=so, dyn_obs=np.zeros((1, n, 2), np.int16), dyn_goal=np.zeros((1, n), np.uint8)), K
