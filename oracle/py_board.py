"""Pure-Python scalar restatement of the createBoard profile (CPU baseline of the board leg).

TEST / BASELINE INFRASTRUCTURE ONLY: imported by tests/ (checked against the golden vectors
the reference produced, tests/golden/board.npz) and by bench.py's board CPU baseline, which
times it on the GPU box's host cores because the reference itself may not travel there.  The
product path never imports this module.

It keeps the reference's per-step structure and cost profile on purpose: a state *list*, one
object per obstacle, ``math.sqrt(math.pow(..))`` distances, ``np.random.ranf`` spawns, and
featureExtractor's numpy calls per obstacle (``np.linalg.norm`` distances, ``np.arccos`` of
clipped dot products of unit vectors, ``np.exp`` social forces), each feature group in its own
loop over the obstacle list, exactly as many of them per step as the reference makes:

* ``PyBoard.reset``        <- createBoard.reset        ballenv_pygame.py:460-513 (Obstacle :21-50,
                                                      generate_randomval :454-457)
* ``PyBoard.step``         <- createBoard.step         ballenv_pygame.py:650-675
* ``PyBoard.calc_reward``  <- createBoard.calc_reward  ballenv_pygame.py:680-706 (check_overlap :381-387)
* ``features``             <- featureExtractor         featureExtractor.py:247-265 (calcDistance :36-40,
                              angle_between :43-56, calcOrientationAndVelocity :61-86,
                              densityFeatures :91-112, speedOrientationFeatures :115-130,
                              calcDistanceFromGoal :132-144, relativeGoalPos :146-166,
                              socialForcesFeatures :170-193)

The reference ends featureExtractor with a torch FloatTensor (``.to(device)``); here the
20 features come back as an f32 numpy row.  Module constants follow ballenv_pygame.py:8-16
(100 x 100 field, spawn strips over the whole field).
"""
from __future__ import annotations

import math
import time

import numpy as np

FIELD = 100                                                # _screen_width / _screen_height
ACTIONS = [(0, -1), (1, 0), (0, 1), (-1, 0)]               # createBoard.actionArray (:352-353)


class _Draws:
    """ranf / randint source: a recorded tape (the reference's values in call order) or
    numpy's legacy global generator, as the reference draws."""

    def __init__(self, tape=None):
        self.tape = None if tape is None else [float(v) for v in tape]
        self.pos = 0

    def _next(self):
        v = self.tape[self.pos]
        self.pos += 1
        return v

    def ranf(self):
        return self._next() if self.tape is not None else float(np.random.ranf())

    def randint(self, lo, hi):
        return int(self._next()) if self.tape is not None else int(np.random.randint(lo, hi))


class _Obs:
    """An Obstacle as createBoard.reset builds it: ``Obstacle(static_obstacle_radius)`` passes
    the radius as the id, so rad keeps its default 20 and the velocities are 0 (:24-47)."""
    __slots__ = ("x", "y", "rad", "vel_x", "vel_y")

    def __init__(self, draws):
        self.x = draws.randint(0, FIELD)
        self.y = draws.randint(0, FIELD)
        self.rad, self.vel_x, self.vel_y = 20, 0, 0


class PyBoard:
    def __init__(self, static_obstacles=6, agent_radius=10, static_obstacle_radius=10):
        self.ns, self.agent_radius, self.rad_static = static_obstacles, agent_radius, static_obstacle_radius
        self.goal_threshold = 15
        self.agent_vel = (0, 0)
        self.state, self.obstacle_list = None, []
        self.total_distance = self.old_dist = None
        self.total_reward_accumulated = 0
        self.sensor_readings = None

    @staticmethod
    def distance(p, q):                                    # calculate_distance (:375-379)
        return math.sqrt(math.pow(p[0] - q[0], 2) + math.pow(p[1] - q[1], 2))

    def overlaps(self, p, q, thresh=0):                    # check_overlap (:381-387)
        return not (self.distance(p, q) - thresh > self.rad_static + self.agent_radius)

    def reset(self, draws=None):
        r = draws if draws is not None else _Draws()
        rv = lambda lo, hi: lo + r.ranf() * (hi - lo)      # noqa: E731  generate_randomval
        gx, gy = rv(0, FIELD), rv(0, FIELD)
        ax, ay = rv(0, FIELD), rv(0, FIELD)
        d0 = math.sqrt(math.pow(gx - ax, 2) + math.pow(gy - ay, 2))
        self.old_dist = d0
        while self.distance((gx, gy), (ax, ay)) < 50:
            ax, ay = rv(0, FIELD), rv(0, FIELD)
        self.state = [(ax, ay), (gx, gy), d0]
        self.total_reward_accumulated = 0
        self.obstacle_list = []
        for _ in range(self.ns):
            while True:
                o = _Obs(r)
                if not self.overlaps((o.x, o.y), (ax, ay), 15) and not self.overlaps((o.x, o.y), (gx, gy), 5):
                    self.state.append((o.x, o.y, o.rad))
                    self.obstacle_list.append(o)
                    break
        self.total_distance = self.distance(self.state[0], self.state[1])
        self.sensor_readings = features(self.state, self.obstacle_list, self.agent_vel, self.agent_radius)
        return self.state

    def step(self, action):
        self.old_dist = self.distance(self.state[0], self.state[1])
        nx = min(max(self.state[0][0] + action[0], 0), FIELD)
        ny = min(max(self.state[0][1] + action[1], 0), FIELD)
        self.state[0] = (nx, ny)
        self.state[2] = self.distance(self.state[0], self.state[1])
        reward, done = self.calc_reward()
        self.sensor_readings = features(self.state, self.obstacle_list, self.agent_vel, self.agent_radius)
        np.array(self.state, dtype=object)        # the reference returns np.asarray(self.state) (:675)
        return self.state, reward, done

    def calc_reward(self):
        for o in self.obstacle_list:                      # first hit ends the episode
            if self.overlaps(self.state[0], (o.x, o.y)):
                self.total_reward_accumulated += -1
                return -1, True
        if self.distance(self.state[0], self.state[1]) < self.goal_threshold:
            self.total_reward_accumulated += 1
            return 1, True
        cur = self.distance(self.state[0], self.state[1])
        reward = (self.old_dist - cur) / self.total_distance
        self.total_reward_accumulated += reward
        return reward, False


# ---------------------------------------------------------------- featureExtractor (:36-265)
def _gap(o, agent, rad):                                   # calcDistance: centre distance - both radii
    return np.linalg.norm((o.x - agent[0], o.y - agent[1])) - rad - o.rad


def _unit(v):
    return v / np.linalg.norm(v) if np.linalg.norm(v) > 0 else v


def _angle(v1, v2):
    return np.arccos(np.clip(np.dot(_unit(v1), _unit(v2)), -1.0, 1.0))


def _bins(o, agent, vel):                                  # (orientation bin, relative-speed bin)
    rel_pos = np.asarray([o.x - agent[0], o.y - agent[1]])
    rel_vel = np.asarray([o.vel_x - vel[0], o.vel_y - vel[1]])
    speed = np.linalg.norm(rel_vel)
    sb = 0 if speed < 0.015 else (1 if speed < 0.025 else 2)
    ang = _angle(rel_pos, rel_vel)
    if ang < math.pi / 4:
        return 0, sb
    if math.pi / 4 < ang < math.pi * 3 / 4:
        return 1, sb
    return 2, sb


def features(state, obstacles, vel, rad):
    agent, goal = state[0], state[1]
    dg = math.floor(np.hypot(agent[0] - goal[0], agent[1] - goal[1]) / 5)
    f_goal = np.asarray([min(dg, 5)])
    xi, yi = goal[0] - agent[0], goal[1] - agent[1]
    rel = np.zeros(4)
    ang = _angle([0, 1], (xi, yi))
    if ang < math.pi / 4:
        rel[0] = 1
    elif math.pi / 4 < ang < math.pi * 3 / 4:
        rel[1 if xi > 0 else 3] = 1
    else:
        rel[2] = 1
    dens = np.zeros(3)
    for o in obstacles:
        g = _gap(o, agent, rad)
        dens[2] += g < 1000
        dens[1] += g < 230
        dens[0] += g < 101
    orsp = np.zeros([3, 3])
    for o in obstacles:
        i, j = _bins(o, agent, vel)
        orsp[i, j] += 1
    soc = np.zeros(3)
    for o in obstacles:                                    # a = 1, b = 10, lambda = 2, threshold 1
        ob, _ = _bins(o, agent, vel)
        psi = _angle(np.asarray([o.x - agent[0], o.y - agent[1]]), np.asarray([o.vel_x - vel[0], o.vel_y - vel[1]]))
        fexp = np.exp(-_gap(o, agent, rad) / 10)
        nij = _gap(o, agent, rad)
        f = fexp * nij * (2 + 0.5 * (1 - 2) * (1 + np.cos(psi)))
        if f > 1:
            soc[ob] += f
    return np.concatenate((f_goal, rel, dens, orsp.reshape(9), soc)).astype(np.float32)


# ---------------------------------------------------------------- CPU baseline
def run_baseline(seconds: float, seed: int = 0, static_obstacles: int = 6, time_limit: int = 1000):
    """Single env, uniform random actionArray moves, reset on done or at the time limit
    (the bench's GPU board leg: same profile, 6 statics, TimeLimit 1000).  step() includes
    featureExtractor, as the reference's does.  Returns (env_steps, elapsed_seconds)."""
    np.random.seed(seed)
    arng = np.random.RandomState(seed + 1)
    b = PyBoard(static_obstacles)
    b.reset()
    steps = t = 0
    t0 = time.perf_counter()
    deadline = t0 + seconds
    while True:
        for _ in range(32):
            _, _, done = b.step(ACTIONS[arng.randint(4)])
            steps += 1
            t += 1
            if done or t >= time_limit:
                b.reset()
                t = 0
        if time.perf_counter() >= deadline:
            break
    return steps, time.perf_counter() - t0


def _worker(args):
    seconds, seed, ns = args
    return run_baseline(seconds, seed, ns)
