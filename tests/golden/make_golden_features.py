"""Golden vectors for the sibling observation formats, made by
RUNNING the reference's own functions (AST-extracted, nothing copied into the repo):

* ``prep_state2`` of examples/ball_env_reinforce.py:130-172 (+ ``block_to_arrpos``
  :169-172): the 29-input block-count encoding -- quadrant one-hot, the agent's own
  cell set, and per obstacle +1 in its 20-px block of a 5x5 grid;
* ``prep_state4`` of examples/potential_fields_modified.py:66-93: the W x W window
  without the quadrant (the potential-field planners' variant), evaluated with a
  reference BallEnv as ``env.unwrapped`` (same gym/numpy shims as make_golden.py).

``prep_state2`` indexes ``ref_state[4+pos]`` with an integral FLOAT (py3 true division
makes ``x_dist/abs(x_dist)`` a float), which numpy >= 1.12 rejects; older numpy took it
as the integer.  The fixture restores that behaviour with an ndarray subclass whose
``__getitem__``/``__setitem__`` accept integral floats (the values are exact integers),
the same kind of shim as make_golden.py's ragged-array proxy.

Writes tests/golden/features.npz.  Run:  python tests/golden/make_golden_features.py
"""
import ast
import math
import os
import sys
from types import SimpleNamespace

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from make_golden import DEFAULT_ARGS, REF, load_reference, make_env  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))


def _top_level_defs(src, names):
    """Source of the named top-level functions (for files that are not Python 3 as a
    whole, e.g. potential_fields_modified.py has py2 print statements elsewhere)."""
    lines = src.splitlines()
    chunks = []
    for i, ln in enumerate(lines):
        if any(ln.startswith(f"def {n}(") for n in names):
            j = i + 1
            while j < len(lines) and (not lines[j].strip() or lines[j][0] in " \t#"):
                j += 1
            chunks.append("\n".join(lines[i:j]).expandtabs(4))
    return "\n\n".join(chunks)


def extract(path, names, g):
    src = open(os.path.join(REF, path)).read()
    try:
        tree = ast.parse(src)
    except SyntaxError:
        tree = ast.parse(_top_level_defs(src, names))
    fns = [n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name in names]
    assert len(fns) == len(names), [n.name for n in fns]
    exec(compile(ast.Module(body=fns, type_ignores=[]), path, "exec"), g)
    return [g[n] for n in names]


def random_cases(rng, n, max_obs=18, span=75):
    agent = np.zeros((n, 2), np.int32)
    goal = np.zeros((n, 2), np.int32)
    obst = np.zeros((n, max_obs, 2), np.int32)
    nobs = np.zeros(n, np.int32)
    for i in range(n):
        ax, ay = int(rng.integers(0, 501)), int(rng.integers(0, 501))
        if rng.integers(4) == 0:
            gx, gy = ax + int(rng.integers(-1, 2)) * int(rng.integers(0, 20)), ay + int(rng.integers(-1, 2)) * int(rng.integers(0, 20))
        else:
            gx, gy = int(rng.integers(0, 500)), int(rng.integers(0, 500))
        k = int(rng.integers(0, max_obs + 1))
        for j in range(k):
            m = rng.integers(6)
            if m == 0:        # same column / row as the agent (x_dist or y_dist == 0)
                ox, oy = (ax, ay + int(rng.integers(-span, span + 1))) if rng.integers(2) else \
                         (ax + int(rng.integers(-span, span + 1)), ay)
            elif m == 1:      # block boundaries: |d| in {9, 10, 11, 29, 30, 31, 49, 50, 51, 69, 70, 71}
                b = [9, 10, 11, 29, 30, 31, 49, 50, 51, 69, 70, 71]
                ox = ax + int(rng.choice(b)) * int(rng.choice([-1, 1]))
                oy = ay + int(rng.choice(b)) * int(rng.choice([-1, 1]))
            elif m == 2:
                ox, oy = int(rng.integers(-40, 540)), int(rng.integers(-40, 540))
            else:
                ox, oy = ax + int(rng.integers(-span, span + 1)), ay + int(rng.integers(-span, span + 1))
            obst[i, j] = (ox, oy)
        agent[i] = (ax, ay); goal[i] = (gx, gy); nobs[i] = k
    return agent, goal, obst, nobs


class _FloatIndexArray(np.ndarray):
    """numpy < 1.12 indexing: an integral float index means that integer."""

    @staticmethod
    def _fix(k):
        if isinstance(k, float):
            assert k == int(k)
            return int(k)
        return k

    def __getitem__(self, k):
        return np.ndarray.__getitem__(self, self._fix(k))

    def __setitem__(self, k, v):
        return np.ndarray.__setitem__(self, self._fix(k), v)


class _OldNumpy:
    def zeros(self, *a, **k):
        return np.zeros(*a, **k).view(_FloatIndexArray)

    def __getattr__(self, n):
        return getattr(np, n)


def main():
    mod, _ = load_reference()
    env = make_env(mod, DEFAULT_ARGS)
    g2 = {"np": _OldNumpy(), "math": math}
    prep_state2, _ = extract("examples/ball_env_reinforce.py", ["prep_state2", "block_to_arrpos"], g2)
    gpf = {"np": np, "math": math, "env": SimpleNamespace(unwrapped=env)}
    (pf_prep4,) = extract("examples/potential_fields_modified.py", ["prep_state4"], gpf)
    rng = np.random.default_rng(2024)
    out = {}
    agent, goal, obst, nobs = random_cases(rng, 1500)
    blocks = np.zeros((len(agent), 29), np.uint8)
    for i in range(len(agent)):
        state = [tuple(agent[i]), tuple(goal[i]), 0.0] + [tuple(p) for p in obst[i, :nobs[i]]]
        r = np.asarray(prep_state2(state))
        assert (r == np.round(r)).all() and r.max() < 256
        blocks[i] = r.astype(np.uint8)
    out.update(blocks_agent=agent, blocks_goal=goal, blocks_obst=obst, blocks_nobs=nobs, blocks_obs=blocks)
    for W in (5, 10):
        agent, goal, obst, nobs = random_cases(rng, 400, span=25 + W + 6)
        win = np.zeros((len(agent), W * W), np.uint8)
        for i in range(len(agent)):
            state = [tuple(agent[i]), tuple(goal[i]), 0.0] + [tuple(p) for p in obst[i, :nobs[i]]]
            win[i] = pf_prep4(state, W).astype(np.uint8)
        out.update({f"pf{W}_agent": agent, f"pf{W}_goal": goal, f"pf{W}_obst": obst, f"pf{W}_nobs": nobs,
                    f"pf{W}_obs": win})
    np.savez_compressed(os.path.join(OUT, "features.npz"), **out)
    print("blocks: cells lit", int((blocks[:, 4:] > 0).sum()), "max count", int(blocks.max()),
          "| pf windows lit", {W: int(out[f'pf{W}_obs'].sum()) for W in (5, 10)})


if __name__ == "__main__":
    main()
