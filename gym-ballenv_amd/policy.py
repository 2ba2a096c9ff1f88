"""The reference's A2C Policy(W) and its batched, on-GPU select_action.

Reference (examples/ball_cnn_ac3.py):
* ``Policy``            :109-146  fc1 (4+W*W -> H) -> relu -> action_head (H -> 9, softmax) / value_head (H -> 1);
                                  H = 128 at W=5, 208 at W=10
* ``select_action``     :210-220  probs, value = policy(state); a ~ Categorical(probs);
                                  saved (log_prob(a), value)
* the rollout loop      :573-600  one env, ``prep_state4`` + ``.to(device)`` + ``.item()`` per step

``HipPolicy`` runs that select_action for every env of a ``BatchedBallEnv`` in
one launch of the hand-written kernel in csrc/policy.hip (libballenv.so,
``be_policy_act``), straight from the u8 obs the step kernel wrote: no host
round trip per step, so a whole rollout captures into one HIP graph
(see ``rollout.py``).  ``torch_select_action`` is the same computation in
plain PyTorch fp32 -- the numerics reference of the tests and the
``backend="torch"`` rollout.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Optional

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _abi

HIDDEN = {5: 128, 10: 208}   # ball_cnn_ac3.py:115-119


class Policy(nn.Module):
    """ball_cnn_ac3.py:109-146 (the same parameter names, so its state_dicts load)."""

    def __init__(self, window: int, hidden: Optional[int] = None, num_actions: int = 9):
        super().__init__()
        if hidden is None:
            if window not in HIDDEN:
                raise ValueError(f"the reference defines Policy hidden sizes for W in {sorted(HIDDEN)}; pass hidden=")
            hidden = HIDDEN[window]
        self.window, self.hidden_layer = window, hidden
        self.fc1 = nn.Linear(4 + window * window, hidden)
        self.action_head = nn.Linear(hidden, num_actions)
        self.value_head = nn.Linear(hidden, 1)

    def forward(self, x):
        x = F.relu(self.fc1(x))
        return F.softmax(self.action_head(x), dim=-1), self.value_head(x)

    @classmethod
    def from_npz(cls, path: str, window: int) -> "Policy":
        """Weights from a fixture written by tests/golden/make_policy_fixture.py."""
        d = np.load(path, allow_pickle=False)
        pol = cls(window, hidden=d["fc1_weight"].shape[0], num_actions=d["action_head_weight"].shape[0])
        pol.load_state_dict({k: torch.from_numpy(d[k.replace(".", "_")]) for k in pol.state_dict()})
        return pol


def reference_weights(window: int) -> Optional[str]:
    """Path of the committed fixture of the reference's trained Policy(W), if any."""
    p = os.path.join(os.path.dirname(os.path.dirname(os.path.realpath(__file__))), "tests", "golden",
                     f"policy_w{window}.npz")
    return p if os.path.exists(p) else None


def torch_select_action(policy: Policy, obs: torch.Tensor, u: torch.Tensor):
    """select_action (ball_cnn_ac3.py:210-220) for a batch, fp32, with the draw
    ``a = #{j : cdf_j <= u}`` from given uniforms ``u`` (N,) -- the rule the HIP
    kernel uses.  Returns (action int64, log_prob, value, probs)."""
    probs, value = policy(obs.float())
    cdf = probs.cumsum(-1)
    a = (cdf <= u.unsqueeze(-1)).sum(-1)
    nz = torch.arange(probs.shape[-1], device=probs.device).expand_as(probs).masked_fill(probs <= 0, 0)
    a = torch.minimum(a, nz.max(-1).values)
    logp = torch.log(probs.gather(-1, a.unsqueeze(-1))).squeeze(-1)
    return a, logp, value.squeeze(-1), probs


class HipPolicy:
    """``be_policy_act`` bound to one BatchedBallEnv (same device, N, W).

    ``load(policy)`` packs the module's current fp32 weights on the device (one
    small kernel, stream-ordered, graph-capturable) -- call it again after an
    optimiser step.  ``act()`` writes ``action`` (N,) u8, ``log_prob`` and
    ``value`` (N,) f32 and, if ``probs=True``, ``probs`` (N, A) f32.
    """

    def __init__(self, env, policy: Optional[Policy] = None, hidden: Optional[int] = None, num_actions: int = 9,
                 probs: bool = False, seed: int = 0x5E1EC7):
        self.env = env
        self._lib = _abi.lib()
        if policy is not None:
            hidden, num_actions = policy.hidden_layer, policy.action_head.out_features
        elif hidden is None:
            hidden = HIDDEN.get(env.window)
        if hidden is None:
            raise ValueError("pass hidden= for this window size")
        self.hidden, self.num_actions, self.seed = int(hidden), int(num_actions), int(seed)
        dev, N = env.device, env.num_envs
        self.action = torch.zeros(N, dtype=torch.uint8, device=dev)
        self.log_prob = torch.zeros(N, dtype=torch.float32, device=dev)
        self.value = torch.zeros(N, dtype=torch.float32, device=dev)
        self.probs = torch.zeros(N, self.num_actions, dtype=torch.float32, device=dev) if probs else None
        self._out = _abi.BeActOut(self.action.data_ptr(), self.log_prob.data_ptr(), self.value.data_ptr(),
                                  None if self.probs is None else self.probs.data_ptr())
        h = C.c_void_p()
        _abi.check(self._lib.be_policy_create(env._ctx, self.hidden, self.num_actions, C.byref(h)), env._ctx)
        self._h = h
        self._weights = None
        if policy is not None:
            self.load(policy)

    def load(self, policy: Policy) -> None:
        dev = self.env.device
        ws = [t.detach().to(device=dev, dtype=torch.float32).contiguous() for t in
              (policy.fc1.weight, policy.fc1.bias, policy.action_head.weight, policy.action_head.bias,
               policy.value_head.weight, policy.value_head.bias)]
        if ws[0].shape != (self.hidden, self.env.obs_dim) or ws[2].shape != (self.num_actions, self.hidden):
            raise ValueError("policy shape does not match this HipPolicy")
        _abi.check(self._lib.be_policy_load(self._h, *[w.data_ptr() for w in ws], self.env._stream()), self.env._ctx)
        self._weights = ws          # keep alive until the packing kernel has run

    @property
    def packed_bytes(self) -> int:
        return int(self._lib.be_policy_bytes(self._h))

    def act(self, obs: Optional[torch.Tensor] = None, seed: Optional[int] = None):
        """select_action for every env from ``obs`` (default: the env's u8 obs buffer)."""
        obs = self.env.obs if obs is None else obs
        if obs.dtype != torch.uint8 or tuple(obs.shape) != (self.env.num_envs, self.env.obs_dim) or \
                not obs.is_contiguous() or obs.device != self.env.device:
            raise ValueError("obs must be the (N, 4+W*W) contiguous u8 window obs on the env's device")
        s = self.seed if seed is None else int(seed)
        _abi.check(self._lib.be_policy_act(self._h, C.byref(self.env._st), obs.data_ptr(), C.byref(self._out),
                                           s & (2**64 - 1), self.env._stream()), self.env._ctx)
        return self.action, self.log_prob, self.value, self.probs

    def close(self) -> None:
        if getattr(self, "_h", None) is not None:
            torch.cuda.synchronize(self.env.device)
            self._lib.be_policy_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
