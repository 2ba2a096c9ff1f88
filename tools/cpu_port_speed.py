"""SURVEY 8(d) check of the CPU baselines: the scalar ports that bench.py times on the GPU box
(oracle/py_ballenv.py, oracle/py_board.py) must run within +-25 % of the reference's own code on
the same host, or the reported CPU baseline would flatter (or slight) the GPU.

Runs ONLY in the build container (it imports the reference from /root/reference with the
shims of tests/golden/make_golden*.py; nothing of the reference is copied).  Single process,
one core, REPS back-to-back reference / port pairs, median of the per-pair ratios:

* BallEnv.step + prep_state4 (ballenv_env.py:232-289, ball_cnn_ac3.py:384-412), 13 static +
  5 dynamic obstacles, random 9-way actions, reset on done / 1000 steps, W = 5 and W = 10;
  SURVEY 8(d) recorded 2.9 k / 0.87 k env-steps/s for the reference on this host;
* createBoard.step incl. featureExtractor (ballenv_pygame.py:650-706, featureExtractor.py:247-265),
  random actionArray moves, reset on done / 1000 steps, 13 statics (1 280
  env-steps/s) and 6 statics (bench.py's board leg).

    python tools/cpu_port_speed.py [--seconds 2] [--reps 9] > profiles/r04_cpu_port_speed.json
"""
import argparse
import contextlib
import io
import json
import os
import statistics
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))

import make_golden as mg            # noqa: E402  (reference loader + shims)
import make_golden_board as mgb     # noqa: E402
from oracle import py_ballenv, py_board   # noqa: E402

MOVES = py_ballenv.MOVE_LIST


def ref_ballenv_rate(mod, W, seconds, seed):
    env = mg.make_env(mod, mg.DEFAULT_ARGS)
    prep4 = mg.load_prep_state(env)
    np.random.seed(seed)
    arng = np.random.RandomState(seed + 1)

    def reset():
        env.static_obstacle_list = []
        env.dynamic_obstacle_list = []       # no stale obstacles
        st = env.reset()
        prep4(env.state, W)
        return st

    reset()
    n = t = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        for _ in range(32):
            state, _, done, _ = env.step(MOVES[arng.randint(9)])
            prep4(state, W)
            n += 1
            t += 1
            if done or t >= 1000:
                reset()
                t = 0
    return n / (time.perf_counter() - t0)


def port_ballenv_rate(W, seconds, seed):
    n, el = py_ballenv.run_baseline(W, seconds, seed)
    return n / el


def ref_board_rate(bp, fe, ns, seconds, seed):
    np.random.seed(seed)
    arng = np.random.RandomState(seed + 1)
    with contextlib.redirect_stdout(io.StringIO()):      # createBoard.__init__ prints
        b = bp.createBoard(static_obstacles=ns, display=False)
    b.reset()
    n = t = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        for _ in range(32):
            _, _, done, _ = b.step(np.asarray(mgb.ACTIONS[arng.randint(4)]))
            n += 1
            t += 1
            if done or t >= 1000:
                b.obstacle_list = []
                b.static_obstacle_list = []
                b.reset()
                t = 0
    return n / (time.perf_counter() - t0)


def port_board_rate(ns, seconds, seed):
    n, el = py_board.run_baseline(seconds, seed, ns)
    return n / el


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=2.0)
    ap.add_argument("--reps", type=int, default=9)
    a = ap.parse_args()
    mod, _ = mg.load_reference()
    bp, fe, _ = mgb.load()
    cases = []
    for W in (5, 10):
        cases.append((f"ballenv W={W}", lambda s, r, W=W: ref_ballenv_rate(mod, W, a.seconds, s),
                      lambda s, r, W=W: port_ballenv_rate(W, a.seconds, s),
                      {5: 2900.0, 10: 870.0}[W]))
    for ns in (13, 6):
        cases.append((f"createBoard statics={ns}", lambda s, r, ns=ns: ref_board_rate(bp, fe, ns, a.seconds, s),
                      lambda s, r, ns=ns: port_board_rate(ns, a.seconds, s), 1280.0 if ns == 13 else None))
    out = {"what": "single-core env-steps/s, reference code vs the scalar CPU ports bench.py times (interleaved, "
                   f"{a.reps} back-to-back pairs of {a.seconds:.0f}-s runs; port_over_reference = median of the per-pair "
                   "ratios, the rates = medians of the runs)",
           "host": os.uname().nodename, "cpu": _cpu_model(), "cases": []}
    for name, ref, port, recorded in cases:
        rr, pr = [], []
        for rep in range(a.reps):        # back-to-back pairs: the host's load drifts between pairs
            rr.append(ref(100 + rep, rep))
            pr.append(port(100 + rep, rep))
        r, p = statistics.median(rr), statistics.median(pr)
        ratio = statistics.median([y / x for x, y in zip(rr, pr)])
        row = {"case": name, "reference": r, "port": p, "port_over_reference": ratio,
               "within_25pct": abs(ratio - 1.0) <= 0.25, "reference_runs": rr, "port_runs": pr}
        if recorded:
            row["recorded_reference"] = recorded
            row["port_over_recorded"] = p / recorded
        out["cases"].append(row)
        print(json.dumps(row), file=sys.stderr, flush=True)
    print(json.dumps(out, indent=1))


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


if __name__ == "__main__":
    main()
