"""INTEGRATION.md's ctypes stub is runnable and agrees with BatchedBallEnv."""
import os
import re

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def stub_source():
    txt = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    blocks = re.findall(r"```python\n(.*?)```", txt, flags=re.S)
    return next(b for b in blocks if "be_create" in b)


def test_stub_parses():
    compile(stub_source(), "INTEGRATION.md", "exec")


@pytest.mark.gpu
def test_ctypes_stub_matches_batched_env(gpu, monkeypatch):
    import gym_ballenv_amd as gb
    monkeypatch.chdir(ROOT)
    ns = {}
    exec(compile(stub_source(), "INTEGRATION.md", "exec"), ns)
    torch.cuda.synchronize()
    env = gb.BatchedBallEnv(ns["N"], ns["W"], device="cuda:0")
    env.reset()
    obs, reward, done, _ = env.step(ns["actions"])
    assert np.array_equal(obs.cpu().numpy(), ns["obs"].cpu().numpy())
    assert np.array_equal(reward.cpu().numpy(), ns["reward"].cpu().numpy())
    assert np.array_equal(done.cpu().numpy(), ns["done"].cpu().numpy().astype(bool))
    env.close()
