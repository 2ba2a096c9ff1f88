"""Pure-Python scalar restatement of the reference hot path (CPU baseline).

TEST / BASELINE INFRASTRUCTURE ONLY: imported by tests/ (checked against the
golden vectors the reference produced) and by bench.py's ``cpu_baseline`` leg,
which times it on the GPU box's host cores because the reference itself may
not travel there.  The product path never imports this module.

It keeps the reference's per-step structure and cost profile on purpose -- a
state *list*, ``math.sqrt(math.pow(..))`` distances, numpy legacy ``randint``
draws, and the W*W*N_obs ``check_overlap`` triple loop of prep_state4:

* ``reset``            <- BallEnv.reset          gym_ballenv/envs/ballenv_env.py:113-167
* ``step``             <- BallEnv.step           ballenv_env.py:232-289
* ``_move_obstacle``   <- move_obstacles         ballenv_env.py:323-353
* ``_reward``          <- calculate_reward       ballenv_env.py:200-229
* ``prep_state4``      <- prep_state4/prep_state2 examples/ball_cnn_ac3.py:330-352, 384-412
"""
from __future__ import annotations

import math
import time

import numpy as np

MOVE_LIST = [(1, 1), (1, -1), (1, 0), (0, 1), (0, -1), (0, 0), (-1, 1), (-1, 0), (-1, -1)]
OBS_MOVES = [(1, 1), (1, -1), (1, 0), (0, 1), (0, -1), (0, 0), (-1, 1), (-1, -1), (-1, -1)]

DEFAULTS = dict(screen_width=500, screen_height=500, strip_obs_x=0, strip_obs_y=20,
                strip_goal_x=500, strip_goal_y=20, strip_agent_x=500, strip_agent_y=10,
                radius_obstacle=20, radius_agent=5, speed_x=1, speed_y=1, threshold_goal=10,
                time_penalty=0, min_spawn_dist=50, num_static=13, num_dynamic=5,
                static_penalty=1, dynamic_penalty=8000, goal_change_step=50, obs_certainty=60,
                goals=[(12, 122), (123, 93), (87, 150), (430, 440), (230, 11)],
                obstacle_speed=[1, 1, 1, 1, 1])


class _Draws:
    """randint source: a recorded tape (parity) or numpy's legacy generator."""

    def __init__(self, tape=None, rng=None):
        self.tape = list(tape) if tape is not None else None
        self.pos = 0
        self.rng = rng if rng is not None else np.random

    def randint(self, lo, hi=None):
        if hi is None:
            lo, hi = 0, lo
        if self.tape is not None:
            v = self.tape[self.pos]
            self.pos += 1
            return int(v)
        return int(self.rng.randint(lo, hi))


class _Wrapped:
    """gym's wrapper as prep_state4 sees it: ``env.unwrapped`` is the BallEnv."""
    __slots__ = ("unwrapped",)

    def __init__(self, env):
        self.unwrapped = env


class PyBallEnv:
    def __init__(self, **cfg):
        c = dict(DEFAULTS)
        c.update(cfg)
        self.c = c
        self.state = None
        self.static = []          # [[x, y], ...]
        self.dyn = []             # [[x, y, goal_index, counter], ...]
        self.total_distance = None
        self.total_reward_accumulated = 0.0
        self.elapsed = 0
        self._env = _Wrapped(self)

    # ballenv_env.py:179-191
    @staticmethod
    def calculate_distance(t1, t2):
        return math.sqrt(math.pow(t1[0] - t2[0], 2) + math.pow(t1[1] - t2[1], 2))

    def check_overlap(self, t1, t2):
        d = self.calculate_distance(t1, t2)
        return not d > (self.c["radius_obstacle"] + self.c["radius_agent"])

    def check_overlap_rect(self, t1, t2, rad):
        return (abs(t1[0] - t2[0]) < rad + self.c["radius_agent"]
                and abs(t1[1] - t2[1]) < rad / 2 + self.c["radius_agent"])

    def reset(self, draws=None):
        c = self.c
        r = draws if draws is not None else _Draws()
        W, H = c["screen_width"], c["screen_height"]
        gx = r.randint(W - c["strip_goal_x"], W)
        gy = r.randint(H - c["strip_goal_y"], H)
        ax = r.randint(0, c["strip_agent_x"])
        ay = r.randint(0, c["strip_agent_y"])
        dist = math.sqrt(math.pow(gx - ax, 2) + math.pow(gy - ay, 2))
        while self.calculate_distance((gx, gy), (ax, ay)) < c["min_spawn_dist"]:
            ax = r.randint(0, c["strip_agent_x"])
            ay = r.randint(0, c["strip_agent_y"])
        self.goal = (gx, gy)
        self.state = [(ax, ay), (gx, gy), dist]
        self.total_reward_accumulated = 0.0
        self.elapsed = 0
        self.static, self.dyn = [], []
        for _ in range(c["num_static"]):
            while True:
                ox = r.randint(c["strip_obs_x"], W - c["strip_obs_x"])
                oy = r.randint(c["strip_obs_y"], H - c["strip_obs_y"])
                if (not self.check_overlap_rect((ox, oy), (ax, ay), c["radius_obstacle"])
                        and not self.check_overlap_rect((ox, oy), (gx, gy), c["radius_obstacle"])):
                    self.static.append([ox, oy])
                    self.state.append((ox, oy))
                    break
        for j in range(c["num_dynamic"]):
            ox = r.randint(c["strip_obs_x"], W - c["strip_obs_x"])
            oy = r.randint(c["strip_obs_y"], H - c["strip_obs_y"])
            self.dyn.append([ox, oy, j, 0])
            self.state.append((ox, oy))
        self.total_distance = self.calculate_distance(self.state[0], self.state[1])
        return self.state

    def set_state(self, agent, goal, prev_dist, total_dist, static, dyn, dyn_goal, counter=0):
        self.goal = tuple(goal)
        self.state = [tuple(agent), tuple(goal), float(prev_dist)]
        self.static = [list(p) for p in static]
        self.dyn = [[p[0], p[1], g, counter] for p, g in zip(dyn, dyn_goal)]
        self.state += [tuple(p) for p in self.static] + [(d[0], d[1]) for d in self.dyn]
        self.total_distance = float(total_dist)
        self.total_reward_accumulated = 0.0

    def _move_obstacle(self, o, j, r):
        c = self.c
        speed = c["obstacle_speed"][j]
        goals = c["goals"]
        if o[3] < c["goal_change_step"]:
            g = goals[o[2]]
            tx, ty = g[0] - o[0], g[1] - o[1]
            if tx != 0 and ty != 0:
                if r.randint(100) < c["obs_certainty"]:
                    o[0] += (tx // abs(tx)) * speed
                    o[1] += (ty // abs(ty)) * speed
                else:
                    i = r.randint(9)
                    o[0] += OBS_MOVES[i][0] * speed
                    o[1] += OBS_MOVES[i][1] * speed
            else:
                i = r.randint(9)
                o[0] += OBS_MOVES[i][0] * speed
                o[1] += OBS_MOVES[i][1] * speed
            o[3] += 1
        else:
            cur = goals[o[2]]
            others = [q for q, g in enumerate(goals) if g != cur]
            o[2] = others[r.randint(len(others))]
            o[3] = 0

    def _reward(self, dist):
        c = self.c
        reward = -c["time_penalty"]
        reward += (self.state_old - dist) / self.total_distance
        done = False
        agent = self.state[0]
        for (ox, oy) in [tuple(p) for p in self.static]:
            done = self.check_overlap(agent, (ox, oy))
            if done:
                return reward - c["static_penalty"], True
        for d in self.dyn:
            done = self.check_overlap(agent, (d[0], d[1]))
            if done:
                return reward - c["dynamic_penalty"], True
        return reward, done

    def step(self, action, draws_per_obstacle=None, rng=None):
        """action: (dx, dy).  draws_per_obstacle: list (per dynamic obstacle) of tapes."""
        c = self.c
        self.state_old = self.state[2]
        x, y = self.state[0]
        nx = x + c["speed_x"] * action[0]
        ny = y + c["speed_y"] * action[1]
        nx = min(max(nx, 0), c["screen_width"])
        ny = min(max(ny, 0), c["screen_height"])
        for j, o in enumerate(self.dyn):
            r = _Draws(draws_per_obstacle[j]) if draws_per_obstacle is not None else _Draws(rng=rng)
            self._move_obstacle(o, j, r)
        gx, gy = self.goal
        dist = math.sqrt(math.pow(gx - nx, 2) + math.pow(gy - ny, 2))
        self.state = [(nx, ny), (gx, gy), dist] + [tuple(p) for p in self.static] + \
                     [(d[0], d[1]) for d in self.dyn]
        goal_flag = dist < c["threshold_goal"]
        reward, obs_flag = self._reward(dist)
        self.total_reward_accumulated += reward
        self.elapsed += 1
        np.array(self.state, dtype=object)   # the reference returns np.array(self.state) (:289)
        return self.state, reward, goal_flag or obs_flag

    def prep_state2(self, state):
        """Quadrant one-hot of the goal relative to the agent (ball_cnn_ac3.py:330-352)."""
        q = np.zeros(4)
        ax, ay = state[0]
        gx, gy = state[1]
        dx, dy = gx - ax, gy - ay
        if dx >= 0 and dy >= 0:
            q[1] = 1
        elif dx < 0 and dy >= 0:
            q[0] = 1
        elif dx < 0 and dy < 0:
            q[3] = 1
        else:
            q[2] = 1
        return q

    def prep_state4(self, state, window):
        """Quadrant one-hot ++ W*W occupancy window (f64 0/1 numpy row, as the reference builds
        it before its torch conversion).  Like the reference it reaches the env's settings and
        check_overlap through ``env.unwrapped`` inside the cell x obstacle loop."""
        env = self._env
        out = np.zeros(4 + window * window)
        out[0:4] = self.prep_state2(state)
        counter = 4
        ax, ay = state[0]
        step_x, step_y = env.unwrapped.c["speed_x"], env.unwrapped.c["speed_y"]
        start_x = ax - env.unwrapped.c["speed_x"] * int(window / 2)
        start_y = ay - env.unwrapped.c["speed_y"] * int(window / 2)
        cur_y = start_y
        for r in range(window):
            for cc in range(window):
                cur_x = start_x + step_x * cc
                for i in range(3, len(state)):
                    if env.unwrapped.check_overlap((cur_x, cur_y), state[i]):
                        out[counter] = 1
                        break
                counter += 1
            cur_y = start_y + step_y * r
        return out


def run_baseline(window: int, seconds: float, seed: int = 0, time_limit: int = 1000):
    """Single env, uniform random 9-way actions, reset on done or at the time limit.

    Returns (env_steps, elapsed_seconds).  Mirrors the ball_cnn_ac3.py rollout
    minus the policy: step() then prep_state4() every step.
    """
    np.random.seed(seed)
    arng = np.random.RandomState(seed + 1)
    env = PyBallEnv()
    state = env.reset()
    env.prep_state4(state, window)
    steps = 0
    t0 = time.perf_counter()
    deadline = t0 + seconds
    while True:
        for _ in range(64):
            a = MOVE_LIST[arng.randint(9)]
            state, reward, done = env.step(a)
            env.prep_state4(state, window)
            steps += 1
            if done or env.elapsed >= time_limit:
                state = env.reset()
                env.prep_state4(state, window)
        if time.perf_counter() >= deadline:
            break
    return steps, time.perf_counter() - t0


def _worker(args):
    window, seconds, seed = args
    return run_baseline(window, seconds, seed)


def run_baseline_parallel(window: int, seconds: float, procs: int):
    """One process per core; returns (total_steps, max_elapsed, per_proc_rates)."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    with ctx.Pool(procs) as pool:
        res = pool.map(_worker, [(window, seconds, 1000 + i) for i in range(procs)])
    total = sum(s for s, _ in res)
    el = max(t for _, t in res)
    return total, el, [s / t for s, t in res]


def run_rollout(window: int, steps: int, seed: int = 0, time_limit: int = 1000):
    """BASELINE config 1: ONE single-env rollout of exactly `steps` random-action steps
    (step + prep_state4, reset on done).  Returns (steps, elapsed_seconds)."""
    np.random.seed(seed)
    arng = np.random.RandomState(seed + 1)
    env = PyBallEnv()
    t0 = time.perf_counter()
    state = env.reset()
    env.prep_state4(state, window)
    for _ in range(steps):
        state, reward, done = env.step(MOVE_LIST[arng.randint(9)])
        env.prep_state4(state, window)
        if done or env.elapsed >= time_limit:
            state = env.reset()
            env.prep_state4(state, window)
    return steps, time.perf_counter() - t0
