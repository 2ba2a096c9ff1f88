"""Diagnostics build (-DBE_STEP4): the four-lanes-per-env proxy against step2_kernel -- obs,
reward, done, truncated and the state must match bit for bit over 200 default-config steps
(its statistics fold is left out)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import gym_ballenv_amd as gb  # noqa: E402

N, W = 65536, 10
envs = []
for lpe in ("2", "4"):
    os.environ["BALLENV_STEP_LPE"] = lpe
    envs.append(gb.BatchedBallEnv(N, W, gb.EnvConfig(), device="cuda:0", seed=5))
print([e.kernel_name("step") for e in envs])
lens = torch.from_numpy(np.random.default_rng(1).integers(0, 1000, N).astype(np.int32)).cuda()
for e in envs:
    e.reset()
    e.ep_len.copy_(lens)
acts = envs[0].sample_actions(200, seed=3)
nd = 0
for t in range(200):
    r = [e.step(acts[t]) for e in envs]
    for a, b in zip(r[0][:3], r[1][:3]):
        assert torch.equal(a, b), t
    assert torch.equal(r[0][3]["truncated"], r[1][3]["truncated"]), t
    nd += int(r[0][2].sum())
s0, s1 = envs[0].state_dict(), envs[1].state_dict()
for k in s0:
    assert torch.equal(s0[k], s1[k]), k
print(f"4-lane proxy == step2_kernel over 200 steps ({nd} dones)")
