"""Minimal gym.spaces stand-ins (gym is not a dependency of this package).

They carry what callers of BallEnv read: ``Discrete.n`` (ball_cnn_ac3.py:485
reads ``env.action_space.n``) and ``Box.shape/low/high``.
"""
from __future__ import annotations

import numpy as np


class Discrete:
    def __init__(self, n: int):
        self.n = int(n)
        self.shape = ()
        self.dtype = np.int64

    def contains(self, x) -> bool:
        try:
            return 0 <= int(x) < self.n
        except (TypeError, ValueError):
            return False

    def sample(self, rng=None) -> int:
        rng = rng or np.random
        return int(rng.randint(self.n))

    def __repr__(self):
        return f"Discrete({self.n})"

    def __eq__(self, other):
        return isinstance(other, Discrete) and other.n == self.n


class Box:
    def __init__(self, low, high, shape=None, dtype=np.float32):
        if shape is None:
            low, high = np.asarray(low, dtype), np.asarray(high, dtype)
            shape = low.shape
        self.shape = tuple(shape)
        self.low = np.broadcast_to(np.asarray(low, dtype), self.shape)
        self.high = np.broadcast_to(np.asarray(high, dtype), self.shape)
        self.dtype = dtype

    def contains(self, x) -> bool:
        x = np.asarray(x)
        return x.shape == self.shape and bool(np.all(x >= self.low) and np.all(x <= self.high))

    def __repr__(self):
        return f"Box({self.shape})"
