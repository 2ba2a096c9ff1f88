"""Golden vectors for the createBoard physics profile, made by
RUNNING the reference: ``ballenv_pygame.createBoard`` (reset :460-513, step :650-675,
calc_reward :680-706, check_overlap :381-387, Obstacle :21-50) and
``featureExtractor.featureExtractor`` (:247-265) which step() calls every step.

Shims (nothing from the reference is copied into the repository):
* ``pygame``: a stub module (init / time.Clock / display are no-ops; display=False);
* ``featureExtractor`` builds a ``torch.cuda.FloatTensor``: torch is proxied so that
  ``torch.cuda.FloatTensor`` is ``torch.FloatTensor`` and the device is the CPU (SURVEY
  §8(c) step 6);
* numpy >= 1.24 refuses the ragged state list in ``np.array(state)``: an np proxy falls
  back to dtype=object (numpy 1.15 behaviour), as make_golden.py does;
* ``np.random.ranf`` / ``np.random.randint`` calls are recorded in order as a draw tape
  (f64: ranf values, and randint values exactly), so the GPU engine can replay them.

Writes tests/golden/board.npz.  Run:  python tests/golden/make_golden_board.py
"""
import importlib.util
import os
import sys
import types

import numpy as np
import torch

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))
ACTIONS = [(0, -1), (1, 0), (0, 1), (-1, 0)]      # createBoard.actionArray (:352-353)


class _Rand:
    def __init__(self):
        self.log = None

    def ranf(self, *a):
        v = float(np.random.ranf(*a))
        if self.log is not None:
            self.log.append(v)
        return v

    def randint(self, *a, **k):
        v = int(np.random.randint(*a, **k))
        if self.log is not None:
            self.log.append(float(v))
        return v

    def __getattr__(self, n):
        return getattr(np.random, n)


class _Np:
    def __init__(self):
        self.random = _Rand()

    def array(self, x, *a, **k):
        try:
            return np.array(x, *a, **k)
        except ValueError:
            return np.array(x, dtype=object)

    asarray = array

    def __getattr__(self, n):
        return getattr(np, n)


def load():
    pg = types.ModuleType("pygame")
    pg.init = lambda: (6, 0)
    pg.time = types.SimpleNamespace(Clock=lambda: types.SimpleNamespace(tick=lambda *a: 0))
    pg.display = types.SimpleNamespace(set_mode=lambda *a: None, set_caption=lambda *a: None, update=lambda: None)
    sys.modules["pygame"] = pg
    tproxy = types.SimpleNamespace(**{k: getattr(torch, k) for k in ("from_numpy", "device")})
    tproxy.cuda = types.SimpleNamespace(FloatTensor=torch.FloatTensor, is_available=lambda: False)
    sys.path.insert(0, REF)
    spec = importlib.util.spec_from_file_location("featureExtractor", os.path.join(REF, "featureExtractor.py"))
    fe = importlib.util.module_from_spec(spec)
    sys.modules["featureExtractor"] = fe
    spec.loader.exec_module(fe)
    fe.torch = tproxy
    fe.device = torch.device("cpu")
    spec = importlib.util.spec_from_file_location("ref_ballenv_pygame", os.path.join(REF, "ballenv_pygame.py"))
    bp = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bp)
    npx = _Np()
    bp.np = npx
    return bp, fe, npx


def features(fe, board):
    f = fe.featureExtractor(board.state, board.obstacle_list, (board.agent_x_vel, board.agent_y_vel),
                            board.agent_radius)
    return f.numpy().reshape(-1).astype(np.float32)


def rollouts(bp, fe, npx, seeds, steps, Ns, directed=False):
    E, T = len(seeds), steps
    d = dict(seeds=np.array(seeds), reset_tape=np.full((E, 256), np.nan), reset_used=np.zeros(E, np.int32),
             init_agent=np.zeros((E, 2)), init_goal=np.zeros((E, 2)), init_dist=np.zeros(E),
             init_total=np.zeros(E), init_static=np.zeros((E, Ns, 2), np.int32),
             init_feat=np.zeros((E, 20), np.float32),
             actions=np.zeros((E, T), np.uint8), reward=np.zeros((E, T)), done=np.zeros((E, T), np.uint8),
             agent=np.zeros((E, T, 2)), dist=np.zeros((E, T)), ep_return=np.zeros((E, T)),
             feat=np.zeros((E, T, 20), np.float32))
    for e, seed in enumerate(seeds):
        np.random.seed(seed)
        b = bp.createBoard(static_obstacles=Ns, display=False)
        npx.random.log = []
        b.reset()
        tape, npx.random.log = npx.random.log, None
        d["reset_tape"][e, :len(tape)] = tape
        d["reset_used"][e] = len(tape)
        d["init_agent"][e] = b.state[0]; d["init_goal"][e] = b.state[1]
        d["init_dist"][e] = b.state[2]; d["init_total"][e] = b.total_distance
        d["init_static"][e] = [(o.x, o.y) for o in b.obstacle_list]
        d["init_feat"][e] = features(fe, b)
        rng = np.random.RandomState(10_000 + seed)
        for t in range(T):
            if directed and rng.randint(100) < 70:
                ax, ay = b.state[0]
                gx, gy = b.state[1]
                a = (1 if gx > ax else 3) if abs(gx - ax) > abs(gy - ay) else (2 if gy > ay else 0)
            else:
                a = int(rng.randint(4))
            d["actions"][e, t] = a
            state, r, done, _ = b.step(np.asarray(ACTIONS[a]))
            d["reward"][e, t] = r; d["done"][e, t] = bool(done)
            d["agent"][e, t] = state[0]; d["dist"][e, t] = state[2]
            d["ep_return"][e, t] = b.total_reward_accumulated
            d["feat"][e, t] = b.sensor_readings.numpy().reshape(-1)
    return d


def main():
    bp, fe, npx = load()
    d = rollouts(bp, fe, npx, list(range(24)), 120, 6)
    d2 = rollouts(bp, fe, npx, list(range(100, 116)), 200, 10, directed=True)
    np.savez_compressed(os.path.join(OUT, "board.npz"), **{f"a_{k}": v for k, v in d.items()},
                        **{f"b_{k}": v for k, v in d2.items()})
    for nm, x in (("random", d), ("directed", d2)):
        print(nm, "steps", x["done"].size, "done", int(x["done"].sum()), "hits", int((x["reward"] == -1).sum()),
              "goals", int((x["reward"] == 1).sum()), "reset draws max", int(x["reset_used"].max()),
              "social-force nonzero", int((x["feat"][..., 17:] != 0).sum()))


if __name__ == "__main__":
    main()
