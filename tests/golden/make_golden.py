"""Generate the golden vectors under tests/golden/ by RUNNING the reference.

This script runs only in the build container (it needs /root/reference, which
does not exist on the GPU box).  It imports the reference's own Python for the
hot path -- ``gym_ballenv/envs/ballenv_env.py`` (BallEnv.reset/step/
move_obstacles/calculate_reward) and the ``prep_state2``/``prep_state4``
functions of ``examples/ball_cnn_ac3.py`` -- with small shims for packages the
image lacks (gym, and numpy>=1.24's refusal of ragged arrays), exactly as
SURVEY.md §8(c) describes.  Nothing from the reference is copied into the
repository: the outputs written here are data (inputs + expected outputs).

Fixtures written (all ``np.savez_compressed``):

* ``rollouts_default.npz`` -- ball_cnn_ac3.py default config (13 static,
  5 dynamic obstacles), seeded episodes: initial SoA state, action tape, the
  reference's dynamic-obstacle ``randint`` draws per (step, obstacle), and the
  expected reward (f64), done, agent/obstacle positions and the W=5 / W=10
  ``prep_state4`` observations after every step.
* ``rollouts_custom.npz`` -- a non-default config (speeds 1..3, 3 goals, goal
  change every 7 steps, 30 % certainty, other penalties/radii/agent speed and
  spawn strips that make the reset re-sample loop fire) at W=7.
* ``resets.npz`` -- reset() draw tapes (every randint value in call order) and
  the resulting SoA state, default and custom strips.
* ``windows.npz`` -- prep_state4 on random states for W in {1,2,3,4,5,10,21,50}
  and on a non-unit cell step / non-default radii.
* ``crafted.npz`` -- single steps from hand-built states covering goal reach,
  the strict goal boundary, collision boundary (d^2 = 625 vs 626), static-
  before-dynamic penalty order, dynamic-only hits, clamps, goal change, the
  tx==0 / ty==0 random-move branch and the u == threshold draw.

Run:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import ast
import importlib.util
import json
import math
import os
import sys
import types
from types import SimpleNamespace

import numpy as np

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))
MOVE_LIST = [(1, 1), (1, -1), (1, 0), (0, 1), (0, -1), (0, 0), (-1, 1), (-1, 0), (-1, -1)]


# --------------------------------------------------------------------------- shims
def _install_gym_stub():
    if "gym" in sys.modules:
        return
    gym = types.ModuleType("gym")
    gym.Env = object
    spaces = types.ModuleType("gym.spaces")

    class Discrete:
        def __init__(self, n):
            self.n = n

    class Box:
        def __init__(self, low, high, *a, **k):
            self.low, self.high = low, high

    spaces.Discrete, spaces.Box = Discrete, Box
    utils = types.ModuleType("gym.utils")
    seeding = types.ModuleType("gym.utils.seeding")
    seeding.np_random = lambda s=None: (np.random.RandomState(s), s)
    utils.seeding = seeding
    error = types.ModuleType("gym.error")
    gym.spaces, gym.utils, gym.error = spaces, utils, error
    for name, mod in {"gym": gym, "gym.spaces": spaces, "gym.utils": utils,
                      "gym.utils.seeding": seeding, "gym.error": error}.items():
        sys.modules[name] = mod


class _RandomProxy:
    """numpy.random stand-in that records every randint value it returns."""

    def __init__(self):
        self.log = None          # list of (lo, hi, value) or None
        self.owner = None        # current dynamic obstacle index (set by wrapper)

    def randint(self, *a, **k):
        v = int(np.random.randint(*a, **k))
        if self.log is not None:
            lo, hi = (0, a[0]) if len(a) == 1 else (a[0], a[1])
            self.log.append((self.owner, lo, hi, v))
        return v

    def __getattr__(self, n):
        return getattr(np.random, n)


class _NpProxy:
    """numpy stand-in: np.array falls back to dtype=object (numpy 1.15 behaviour)."""

    def __init__(self):
        self.random = _RandomProxy()

    def array(self, x, *a, **k):
        try:
            return np.array(x, *a, **k)
        except ValueError:
            return np.array(x, dtype=object)

    def __getattr__(self, n):
        return getattr(np, n)


def load_reference():
    _install_gym_stub()
    spec = importlib.util.spec_from_file_location(
        "ref_ballenv_env", os.path.join(REF, "gym_ballenv/envs/ballenv_env.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    proxy = _NpProxy()
    mod.np = proxy
    return mod, proxy


def load_prep_state(env):
    """AST-extract prep_state2/prep_state4 from examples/ball_cnn_ac3.py."""
    import torch
    src = open(os.path.join(REF, "examples/ball_cnn_ac3.py")).read()
    tree = ast.parse(src)
    fns = [n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name in ("prep_state2", "prep_state4")]
    g = {"np": np, "torch": torch, "device": torch.device("cpu"),
         "env": SimpleNamespace(unwrapped=env), "math": math}
    exec(compile(ast.Module(body=fns, type_ignores=[]), "ball_cnn_ac3_prep", "exec"), g)
    p4 = g["prep_state4"]

    def prep4(state, W):
        return p4(state, W).numpy().reshape(-1).astype(np.uint8)
    return prep4


# --------------------------------------------------------------------------- env helpers
DEFAULT_ARGS = dict(static_obstacles=13, dynamic_obstacles=5, obstacle_speed=[1, 1, 1, 1, 1],
                    obs_goal_position=['12,122', '123,93', '87,150', '430,440', '230,11'],
                    time_step_for_change=50, rd_th_obs=60, rd_th_agent=80,
                    static_thresholds=[0, 0], dynamic_thresholds=[10, 10],
                    static_penalty=[1, 1], dynamic_penalty=[4000, 8000])

CUSTOM_ARGS = dict(static_obstacles=16, dynamic_obstacles=3, obstacle_speed=[1, 2, 3],
                   obs_goal_position=['50,60', '300,400', '450,20'],
                   time_step_for_change=7, rd_th_obs=30, rd_th_agent=80,
                   static_thresholds=[0, 0], dynamic_thresholds=[10, 10],
                   static_penalty=[2, 3], dynamic_penalty=[10, 500])
# knobs that are env attributes / module constants rather than argparse fields
CUSTOM_ENV = dict(radius_rand_person=12, radius_ctrl_person=4, speedx_ctrl_person=2,
                  speedy_ctrl_person=3, threshold_goal=15)
CUSTOM_STRIPS = dict(_stripagenty=500, _stripgoaly=100)


def make_env(mod, args, env_attrs=None):
    env = mod.BallEnv()
    env.customize_environment(SimpleNamespace(**args))
    for k, v in (env_attrs or {}).items():
        setattr(env, k, v)
    return env


def cfg_json(args, env_attrs=None, strips=None, window=None):
    c = dict(args)
    c.update({"env": env_attrs or {}, "strips": strips or {}, "window": window})
    return json.dumps(c)


def soa_snapshot(env):
    goals = env.obstacle_goal_list
    agent = tuple(int(v) for v in env.state[0])
    st = [(int(o.x), int(o.y)) for o in env.static_obstacle_list]
    dy = [(int(o.x), int(o.y)) for o in env.dynamic_obstacle_list]
    dg = [goals.index(o.curr_goal) for o in env.dynamic_obstacle_list]
    cnt = [int(o.curr_counter) for o in env.dynamic_obstacle_list]
    for o in env.static_obstacle_list + env.dynamic_obstacle_list:
        assert float(o.x) == int(o.x) and float(o.y) == int(o.y)
    return dict(agent=agent, goal=(int(env.goal_x), int(env.goal_y)), prev_dist=float(env.state[2]),
                total_dist=float(env.total_distance), static=st, dyn=dy, dyn_goal=dg, counter=cnt)


def fresh_reset(env, proxy):
    # clear the lists so stale obstacles do not consume draws
    env.static_obstacle_list = []
    env.dynamic_obstacle_list = []
    proxy.random.log = []
    proxy.random.owner = None
    env.reset()
    draws = [v for (_, _, _, v) in proxy.random.log]
    proxy.random.log = None
    return draws


def install_move_recorder(env, proxy):
    orig = env.move_obstacles
    index = {}

    def wrapped(obstacle):
        proxy.random.owner = index[id(obstacle)]
        return orig(obstacle)
    env.move_obstacles = wrapped

    def refresh():
        index.clear()
        for j, o in enumerate(env.dynamic_obstacle_list):
            index[id(o)] = j
    return refresh


def rollout_fixture(mod, proxy, args, seeds, steps, windows, env_attrs=None, strips=None,
                    directed=None):
    strips = strips or {}
    saved = {k: getattr(mod, k) for k in strips}
    for k, v in strips.items():
        setattr(mod, k, v)
    try:
        env = make_env(mod, args, env_attrs)
        prep4 = load_prep_state(env)
        refresh = install_move_recorder(env, proxy)
        E, T = len(seeds), steps
        Ns, Nd = args["static_obstacles"], args["dynamic_obstacles"]
        F = {W: 4 + W * W for W in windows}
        d = dict(seeds=np.array(seeds, np.int64),
                 init_agent=np.zeros((E, 2), np.int32), init_goal=np.zeros((E, 2), np.int32),
                 init_prev_dist=np.zeros(E), init_total_dist=np.zeros(E),
                 init_static=np.zeros((E, Ns, 2), np.int32), init_dyn=np.zeros((E, Nd, 2), np.int32),
                 init_dyn_goal=np.zeros((E, Nd), np.int32),
                 actions=np.zeros((E, T), np.uint8), tape=np.full((E, T, Nd, 2), -1, np.int16),
                 reward=np.zeros((E, T)), done=np.zeros((E, T), np.uint8),
                 agent=np.zeros((E, T, 2), np.int32), dyn=np.zeros((E, T, Nd, 2), np.int32),
                 dyn_goal=np.zeros((E, T, Nd), np.int32), ep_return=np.zeros((E, T)))
        for W in windows:
            d[f"init_obs{W}"] = np.zeros((E, F[W]), np.uint8)
            d[f"obs{W}"] = np.zeros((E, T, F[W]), np.uint8)
        for e, seed in enumerate(seeds):
            np.random.seed(seed)
            fresh_reset(env, proxy)
            refresh()
            s = soa_snapshot(env)
            assert all(c == 0 for c in s["counter"])
            d["init_agent"][e] = s["agent"]; d["init_goal"][e] = s["goal"]
            d["init_prev_dist"][e] = s["prev_dist"]; d["init_total_dist"][e] = s["total_dist"]
            if Ns:
                d["init_static"][e] = s["static"]
            if Nd:
                d["init_dyn"][e] = s["dyn"]; d["init_dyn_goal"][e] = s["dyn_goal"]
            for W in windows:
                d[f"init_obs{W}"][e] = prep4(env.state, W)
            arng = np.random.RandomState(100_000 + seed)   # never touches the global stream
            use_dir = directed is not None and e in directed
            for t in range(T):
                if use_dir and arng.randint(100) < 85:
                    ax, ay = env.state[0]
                    dx = int(np.sign(env.goal_x - ax)); dy = int(np.sign(env.goal_y - ay))
                    a = MOVE_LIST.index((dx, dy))
                else:
                    a = int(arng.randint(9))
                d["actions"][e, t] = a
                proxy.random.log = []
                state, reward, done, _ = env.step(MOVE_LIST[a])
                log, proxy.random.log = proxy.random.log, None
                cnt = [0] * Nd
                for (j, lo, hi, v) in log:
                    assert j is not None
                    d["tape"][e, t, j, cnt[j]] = v
                    cnt[j] += 1
                s = soa_snapshot(env)
                d["reward"][e, t] = reward; d["done"][e, t] = bool(done)
                d["agent"][e, t] = s["agent"]
                if Nd:
                    d["dyn"][e, t] = s["dyn"]; d["dyn_goal"][e, t] = s["dyn_goal"]
                d["ep_return"][e, t] = env.total_reward_accumulated
                for W in windows:
                    d[f"obs{W}"][e, t] = prep4(state, W)
        d["config"] = np.array(cfg_json(args, env_attrs, strips))
        return d
    finally:
        for k, v in saved.items():
            setattr(mod, k, v)


def resets_fixture(mod, proxy, args, seeds, env_attrs=None, strips=None, tape_len=96):
    strips = strips or {}
    saved = {k: getattr(mod, k) for k in strips}
    for k, v in strips.items():
        setattr(mod, k, v)
    try:
        env = make_env(mod, args, env_attrs)
        E = len(seeds)
        Ns, Nd = args["static_obstacles"], args["dynamic_obstacles"]
        d = dict(seeds=np.array(seeds, np.int64), tape=np.full((E, tape_len), -1, np.int16),
                 tape_used=np.zeros(E, np.int32),
                 agent=np.zeros((E, 2), np.int32), goal=np.zeros((E, 2), np.int32),
                 prev_dist=np.zeros(E), total_dist=np.zeros(E),
                 static=np.zeros((E, Ns, 2), np.int32), dyn=np.zeros((E, Nd, 2), np.int32),
                 dyn_goal=np.zeros((E, Nd), np.int32))
        for e, seed in enumerate(seeds):
            np.random.seed(seed)
            draws = fresh_reset(env, proxy)
            assert len(draws) <= tape_len, len(draws)
            d["tape"][e, :len(draws)] = draws
            d["tape_used"][e] = len(draws)
            s = soa_snapshot(env)
            d["agent"][e] = s["agent"]; d["goal"][e] = s["goal"]
            d["prev_dist"][e] = s["prev_dist"]; d["total_dist"][e] = s["total_dist"]
            if Ns:
                d["static"][e] = s["static"]
            if Nd:
                d["dyn"][e] = s["dyn"]; d["dyn_goal"][e] = s["dyn_goal"]
        d["config"] = np.array(cfg_json(args, env_attrs, strips))
        return d
    finally:
        for k, v in saved.items():
            setattr(mod, k, v)


def windows_fixture(mod, Ws, per_w, seed=7, env_attrs=None, max_obs=18):
    env = make_env(mod, DEFAULT_ARGS, env_attrs)
    prep4 = load_prep_state(env)
    rng = np.random.RandomState(seed)
    out = {}
    for W in Ws:
        n = per_w if W <= 21 else max(40, per_w // 10)
        agent = np.zeros((n, 2), np.int32); goal = np.zeros((n, 2), np.int32)
        obst = np.full((n, max_obs, 2), 0, np.int32); nobs = np.zeros(n, np.int32)
        obs = np.zeros((n, 4 + W * W), np.uint8)
        for i in range(n):
            ax, ay = int(rng.randint(0, 501)), int(rng.randint(0, 501))
            mode = rng.randint(4)
            if mode == 0:       # goal exactly on an axis / same point (quadrant ties)
                gx = ax + int(rng.randint(-1, 2)) * int(rng.randint(0, 30))
                gy = ay + int(rng.randint(-1, 2)) * int(rng.randint(0, 30))
            else:
                gx, gy = int(rng.randint(0, 500)), int(rng.randint(0, 500))
            k = int(rng.randint(0, max_obs + 1))
            span = 25 + W + 6
            pts = []
            for _ in range(k):
                if rng.randint(4) == 0:
                    pts.append((int(rng.randint(-40, 540)), int(rng.randint(-40, 540))))
                else:
                    pts.append((ax + int(rng.randint(-span, span + 1)), ay + int(rng.randint(-span, span + 1))))
            state = [(ax, ay), (gx, gy), 0.0] + pts
            agent[i] = (ax, ay); goal[i] = (gx, gy); nobs[i] = k
            if k:
                obst[i, :k] = pts
            obs[i] = prep4(state, W)
        out[f"W{W}_agent"] = agent; out[f"W{W}_goal"] = goal
        out[f"W{W}_obst"] = obst; out[f"W{W}_nobs"] = nobs; out[f"W{W}_obs"] = obs
    out["windows"] = np.array(Ws, np.int32)
    out["env"] = np.array(json.dumps(env_attrs or {}))
    return out


def crafted_fixture(mod, proxy):
    """Single steps from hand-built states."""
    args = DEFAULT_ARGS
    env = make_env(mod, args, None)
    prep4 = load_prep_state(env)
    refresh = install_move_recorder(env, proxy)
    goals = [tuple(int(v) for v in g.split(",")) for g in args["obs_goal_position"]]
    Ns, Nd = 13, 5
    cases = []

    def far(i):   # parking spots far from everything
        return (30 * i + 10, 250 + (i % 3) * 7)

    def add(name, agent, goal, prev, total, statics, dyns, dgoal, counter, action, seed=0):
        cases.append(dict(name=name, agent=agent, goal=goal, prev=prev, total=total,
                          statics=statics, dyns=dyns, dgoal=dgoal, counter=counter,
                          action=action, seed=seed))

    st_far = [far(i) for i in range(Ns)]
    dy_far = [(400 + 15 * j, 60 + 11 * j) for j in range(Nd)]
    g0 = [0, 1, 2, 3, 4]
    # goal reach: moving onto dist 9 (< 10)
    add("goal_reach", (200, 480), (200, 490), 10.0, 480.0, st_far, dy_far, g0, 0, MOVE_LIST.index((0, 1)))
    # strict goal boundary: dist exactly 10 after move -> not done
    add("goal_boundary", (200, 479), (200, 490), 11.0, 480.0, st_far, dy_far, g0, 0, MOVE_LIST.index((0, 1)))
    # static collision at exactly d^2 = 625 (15,20)
    st = list(st_far); st[4] = (215, 120)
    add("static_d625", (199, 99), (300, 490), 400.0, 450.0, st, dy_far, g0, 0, MOVE_LIST.index((1, 1)))
    # no collision at d^2 = 626 (25,1)
    st = list(st_far); st[4] = (225, 101)
    add("static_d626", (199, 99), (300, 490), 400.0, 450.0, st, dy_far, g0, 0, MOVE_LIST.index((1, 1)))
    # dynamic-only hit (obstacle 2 sits on the agent; counter at change step so it does not move)
    dy = list(dy_far); dy[2] = (100, 100)
    add("dynamic_only", (100, 99), (300, 490), 400.0, 450.0, st_far, dy, g0, 50, MOVE_LIST.index((0, 1)))
    # static + dynamic both -> static penalty (statics first)
    st = list(st_far); st[0] = (110, 100)
    add("static_before_dynamic", (100, 99), (300, 490), 400.0, 450.0, st, dy, g0, 50, MOVE_LIST.index((0, 1)))
    # clamps at both borders
    add("clamp_low", (0, 0), (300, 490), 400.0, 450.0, st_far, dy_far, g0, 0, MOVE_LIST.index((-1, -1)))
    add("clamp_high", (500, 500), (300, 490), 400.0, 450.0, st_far, dy_far, g0, 0, MOVE_LIST.index((1, 1)))
    add("clamp_x_only", (500, 250), (300, 490), 400.0, 450.0, st_far, dy_far, g0, 0, MOVE_LIST.index((1, -1)))
    # goal change step for every dynamic obstacle, several seeds
    for s in range(6):
        add(f"goal_change_{s}", (250, 5), (300, 490), 400.0, 450.0, st_far, dy_far, [s % 5] * 5, 50, 5, seed=s)
    # tx == 0 / ty == 0 -> the plain random move branch
    dy = [(goals[j][0], 300 + j) for j in range(Nd)]
    add("tx_zero", (250, 5), (300, 490), 400.0, 450.0, st_far, dy, g0, 3, 5, seed=11)
    dy = [(300 + j, goals[j][1]) for j in range(Nd)]
    add("ty_zero", (250, 5), (300, 490), 400.0, 450.0, st_far, dy, g0, 3, 5, seed=12)
    dy = [goals[j] for j in range(Nd)]
    add("at_goal", (250, 5), (300, 490), 400.0, 450.0, st_far, dy, g0, 3, 5, seed=13)
    # many seeds of generic moving obstacles near the agent (dynamic collisions, windows)
    for s in range(40):
        r = np.random.RandomState(500 + s)
        ax, ay = int(r.randint(30, 470)), int(r.randint(30, 470))
        dy = [(ax + int(r.randint(-28, 29)), ay + int(r.randint(-28, 29))) for _ in range(Nd)]
        st = [(ax + int(r.randint(-60, 61)), ay + int(r.randint(-60, 61))) if r.randint(3) == 0 else far(i)
              for i in range(Ns)]
        add(f"near_{s}", (ax, ay), (int(r.randint(0, 500)), int(r.randint(480, 500))),
            float(r.randint(50, 500)), float(r.randint(470, 700)), st, dy,
            [int(r.randint(5)) for _ in range(Nd)], int(r.randint(0, 51)), int(r.randint(9)), seed=1000 + s)

    E = len(cases)
    d = dict(names=np.array([c["name"] for c in cases]),
             init_agent=np.zeros((E, 2), np.int32), init_goal=np.zeros((E, 2), np.int32),
             init_prev_dist=np.zeros(E), init_total_dist=np.zeros(E),
             init_static=np.zeros((E, Ns, 2), np.int32), init_dyn=np.zeros((E, Nd, 2), np.int32),
             init_dyn_goal=np.zeros((E, Nd), np.int32), init_ep_len=np.zeros(E, np.int32),
             actions=np.zeros(E, np.uint8), tape=np.full((E, Nd, 2), -1, np.int16),
             reward=np.zeros(E), done=np.zeros(E, np.uint8), agent=np.zeros((E, 2), np.int32),
             dyn=np.zeros((E, Nd, 2), np.int32), dyn_goal=np.zeros((E, Nd), np.int32),
             obs5=np.zeros((E, 29), np.uint8), obs10=np.zeros((E, 104), np.uint8))
    for e, c in enumerate(cases):
        np.random.seed(c["seed"])
        env.static_obstacle_list = []; env.dynamic_obstacle_list = []
        env.reset()          # builds obstacle objects with the right penalties etc.
        env.goal_x, env.goal_y = c["goal"]
        for o, p in zip(env.static_obstacle_list, c["statics"]):
            o.x, o.y = p
        for o, p, gi in zip(env.dynamic_obstacle_list, c["dyns"], c["dgoal"]):
            o.x, o.y = p
            o.curr_goal = goals[gi]
            o.curr_counter = c["counter"]
        env.state = [c["agent"], c["goal"], c["prev"]] + [(o.x, o.y) for o in env.obstacle_list]
        env.total_distance = c["total"]
        env.total_reward_accumulated = 0
        refresh()
        d["init_agent"][e] = c["agent"]; d["init_goal"][e] = c["goal"]
        d["init_prev_dist"][e] = c["prev"]; d["init_total_dist"][e] = c["total"]
        d["init_static"][e] = c["statics"]; d["init_dyn"][e] = c["dyns"]
        d["init_dyn_goal"][e] = c["dgoal"]; d["init_ep_len"][e] = c["counter"]
        d["actions"][e] = c["action"]
        proxy.random.log = []
        state, reward, done, _ = env.step(MOVE_LIST[c["action"]])
        log, proxy.random.log = proxy.random.log, None
        cnt = [0] * Nd
        for (j, lo, hi, v) in log:
            d["tape"][e, j, cnt[j]] = v
            cnt[j] += 1
        s = soa_snapshot(env)
        d["reward"][e] = reward; d["done"][e] = bool(done); d["agent"][e] = s["agent"]
        d["dyn"][e] = s["dyn"]; d["dyn_goal"][e] = s["dyn_goal"]
        d["obs5"][e] = prep4(state, 5); d["obs10"][e] = prep4(state, 10)
    d["config"] = np.array(cfg_json(args))
    return d


def main():
    mod, proxy = load_reference()
    default_seeds = list(range(16))
    d = rollout_fixture(mod, proxy, DEFAULT_ARGS, default_seeds, 256, (5, 10))
    # 4 longer goal-directed episodes (85 % greedy) so goal reach and many collisions appear
    d2 = rollout_fixture(mod, proxy, DEFAULT_ARGS, [100, 101, 102, 103], 640, (5, 10),
                         directed={0, 1, 2, 3})
    np.savez_compressed(os.path.join(OUT, "rollouts_default.npz"), **d)
    np.savez_compressed(os.path.join(OUT, "rollouts_directed.npz"), **d2)
    c = rollout_fixture(mod, proxy, CUSTOM_ARGS, list(range(200, 212)), 200, (7,),
                        env_attrs=CUSTOM_ENV, strips=CUSTOM_STRIPS, directed=set(range(9)))
    np.savez_compressed(os.path.join(OUT, "rollouts_custom.npz"), **c)
    r1 = resets_fixture(mod, proxy, DEFAULT_ARGS, list(range(300)))
    r2 = resets_fixture(mod, proxy, CUSTOM_ARGS, list(range(300)), env_attrs=CUSTOM_ENV, strips=CUSTOM_STRIPS)
    np.savez_compressed(os.path.join(OUT, "resets.npz"),
                        **{f"default_{k}": v for k, v in r1.items()},
                        **{f"custom_{k}": v for k, v in r2.items()})
    w = windows_fixture(mod, [1, 2, 3, 4, 5, 10, 21, 50], 400)
    w2 = windows_fixture(mod, [5, 10], 300, seed=9,
                         env_attrs=dict(radius_rand_person=12, radius_ctrl_person=4,
                                        speedx_ctrl_person=2, speedy_ctrl_person=3))
    np.savez_compressed(os.path.join(OUT, "windows.npz"), **w)
    np.savez_compressed(os.path.join(OUT, "windows_custom.npz"), **w2)
    cr = crafted_fixture(mod, proxy)
    np.savez_compressed(os.path.join(OUT, "crafted.npz"), **cr)
    # summary for the record
    def stats(x):
        return dict(steps=int(x["done"].size), done=int(x["done"].sum()),
                    hit_static=int(((x["reward"] < -0.5) & (x["reward"] > -100)).sum()),
                    hit_dyn=int((x["reward"] < -100).sum()))
    print("default", stats(d), "directed", stats(d2), "custom", stats(c))
    print("crafted", list(zip(cr["names"][:16], cr["reward"][:16], cr["done"][:16])))


if __name__ == "__main__":
    main()
