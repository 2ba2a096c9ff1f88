"""On-GPU policy rollouts of a BatchedBallEnv (BASELINE config 5).

The reference's A2C driver (examples/ball_cnn_ac3.py:573-600) runs one env on
the host: per step ``prep_state4`` -> ``.to(device)`` -> ``select_action`` ->
``.item()`` -> ``env.step``, and keeps ``policy.saved_actions`` /
``policy.rewards`` lists for ``finish_episode`` (:222-246).  Here a step of all
N envs is two launches that never leave the GPU:

    be_policy_act   obs (N, 4+W*W) u8  ->  action, log_prob, value   (HipPolicy)
    be_step         action             ->  obs, reward, done          (BatchedBallEnv)

and each launch writes straight into row t of the (T, N) trajectory buffers
(per-step ``be_out`` / ``be_act_out`` structs point into them: no copy
kernels).  ``capture()`` records the T-step loop into HIP graphs, so
``run()`` is one graph replay per chunk with no host work per step.

``backend="fused"`` runs the same T steps as ``be_policy_rollout`` launches of ``chunk``
steps each: select_action and the env step in one kernel, each env's state in
registers and the packed policy in LDS (bit-identical to ``"hip"``).

``backend="torch"`` runs select_action as plain PyTorch fp32 (``Policy`` +
``torch_select_action`` on ``torch.rand`` uniforms) -- the PyTorch-ROCm policy
the BASELINE config names, kept as the comparison point.

``discounted_returns`` is the batched form of finish_episode's return
recursion (:224-227) with episode boundaries (done) cutting the sum;
``a2c_losses`` / ``a2c_update`` are the whole finish_episode (per-episode
return normalisation, policy + value losses) over all envs at once, so a
training loop is rollout (HIP) -> update (torch autograd) -> re-pack (HIP).
"""
from __future__ import annotations

import ctypes as C
from typing import Optional

import torch

from . import _abi
from .policy import HipPolicy, Policy, torch_select_action


class Rollout:
    def __init__(self, env, policy: Policy, horizon: int, backend: str = "hip", record_obs: bool = False,
                 seed: int = 0x5E1EC7, chunk: int = 100):
        if backend not in ("hip", "fused", "torch"):
            raise ValueError("backend must be 'hip', 'fused' or 'torch'")
        self.env, self.policy, self.T, self.backend = env, policy, int(horizon), backend
        dev, N, T = env.device, env.num_envs, self.T
        self.seed = int(seed)
        self.actions = torch.zeros(T, N, dtype=torch.uint8, device=dev)
        self.log_probs = torch.zeros(T, N, dtype=torch.float32, device=dev)
        self.values = torch.zeros(T, N, dtype=torch.float32, device=dev)
        self.rewards = torch.zeros(T, N, dtype=torch.float64, device=dev)
        self.dones = torch.zeros(T, N, dtype=torch.bool, device=dev)
        self.obs = torch.zeros(T + 1, N, env.obs_dim, dtype=torch.uint8, device=dev) if record_obs else None
        self._graphs = []
        self._lib = _abi.lib()
        self.chunk = max(1, int(chunk))
        if backend in ("hip", "fused"):
            self.hp = HipPolicy(env, policy, seed=self.seed)
            self._act_outs = [_abi.BeActOut(self.actions[t].data_ptr(), self.log_probs[t].data_ptr(),
                                            self.values[t].data_ptr(), None) for t in range(T)]
        else:
            self.hp = None
            self.policy = policy.to(dev)     # draws: torch.rand on the default (graph-safe) generator
        o = env._out
        self._step_outs = []
        for t in range(T):
            obs_ptr = self.obs[t + 1].data_ptr() if record_obs else o.obs
            self._step_outs.append(_abi.BeOut(obs_ptr, o.obs_f32, self.rewards[t].data_ptr(),
                                              self.dones[t].data_ptr(), o.truncated, o.terminal_obs,
                                              o.final_return, o.final_len, o.stats))

    def run_fused(self, stream_ptr=None) -> None:
        """The horizon as be_policy_rollout launches of ``chunk`` steps (backend="fused")."""
        env, lib, N, F = self.env, self._lib, self.env.num_envs, self.env.obs_dim
        s = env._stream() if stream_ptr is None else stream_ptr
        self.begin()
        for c0 in range(0, self.T, self.chunk):
            k = min(self.chunk, self.T - c0)
            rec = self.obs[c0 + 1].data_ptr() if self.obs is not None else None
            out = _abi.BeOut(rec, None, self.rewards[c0].data_ptr(), self.dones[c0].data_ptr(), None, None,
                             None, None, env._out.stats)
            act = _abi.BeActOut(self.actions[c0].data_ptr(), self.log_probs[c0].data_ptr(),
                                self.values[c0].data_ptr(), None)
            rc = lib.be_policy_rollout(self.hp._h, C.byref(env._st), env.obs.data_ptr(), env.obs.data_ptr(), k,
                                       C.byref(out), C.byref(act), self.seed & (2**64 - 1), s)
            if rc:
                _abi.check(rc, env._ctx)

    def _obs_t(self, t: int) -> torch.Tensor:
        return self.obs[t] if self.obs is not None else self.env.obs

    def step(self, t: int, stream_ptr=None) -> None:
        """select_action + env step of every env, results into row t."""
        env, lib = self.env, self._lib
        s = env._stream() if stream_ptr is None else stream_ptr
        obs = self._obs_t(t)
        if self.backend == "hip":
            rc = lib.be_policy_act(self.hp._h, C.byref(env._st), obs.data_ptr(), C.byref(self._act_outs[t]),
                                   self.seed & (2**64 - 1), s)
            if rc:
                _abi.check(rc, env._ctx)
        else:
            with torch.no_grad():
                u = torch.rand(env.num_envs, device=env.device)
                a, lp, v, _ = torch_select_action(self.policy, obs, u)
                self.actions[t].copy_(a)
                self.log_probs[t].copy_(lp)
                self.values[t].copy_(v)
        rc = lib.be_step(env._ctx, C.byref(env._st), C.c_void_p(self.actions[t].data_ptr()), None, None,
                         C.byref(self._step_outs[t]), s)
        if rc:
            _abi.check(rc, env._ctx)

    def begin(self) -> None:
        """Make row 0 of the obs record the env's current obs (call after reset)."""
        if self.obs is not None:
            self.obs[0].copy_(self.env.obs)

    def end(self) -> None:
        """With record_obs the steps write obs into the record: leave the last one in env.obs."""
        if self.obs is not None:
            self.env.obs.copy_(self.obs[self.T])

    def run_eager(self) -> None:
        if self.backend == "fused":
            return self.run_fused()
        self.begin()
        for t in range(self.T):
            self.step(t)
        self.end()

    def capture(self, chunk: int = 250) -> None:
        """Record the T steps into HIP graphs of ``chunk`` steps each."""
        dev = self.env.device
        if self.backend == "fused":     # a few launches per horizon: nothing to capture
            self._graphs = []
            return
        if self.backend == "torch":
            # initialise the BLAS handles eagerly: hipBLASLt set-up is not capturable
            with torch.no_grad():
                self.policy(self.env.obs[:64].float())
            torch.cuda.synchronize(dev)
        cap = torch.cuda.Stream(dev)
        self._graphs = []
        for c0 in range(0, self.T, chunk):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=cap):
                sp = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
                for t in range(c0, min(self.T, c0 + chunk)):
                    self.step(t, sp)
            self._graphs.append(g)
        torch.cuda.synchronize(dev)

    def run(self) -> None:
        """Replay the captured horizon (capture() first)."""
        if self.backend == "fused":
            return self.run_fused()
        if not self._graphs:
            raise RuntimeError("capture() first")
        self.begin()
        for g in self._graphs:
            g.replay()
        self.end()

    def discounted_returns(self, gamma: float = 0.99, bootstrap: Optional[torch.Tensor] = None) -> torch.Tensor:
        """R_t = r_t + gamma * R_{t+1} * (1 - done_t), per env (finish_episode, ball_cnn_ac3.py:224-227)."""
        R = torch.zeros(self.env.num_envs, dtype=torch.float64, device=self.env.device) if bootstrap is None \
            else bootstrap.to(torch.float64).clone()
        out = torch.empty_like(self.rewards)
        for t in range(self.T - 1, -1, -1):
            R = self.rewards[t] + gamma * R * (~self.dones[t]).to(torch.float64)
            out[t] = R
        return out

    def close(self) -> None:
        self._graphs = []
        if self.hp is not None:
            self.hp.close()


def a2c_losses(policy: Policy, obs: torch.Tensor, actions: torch.Tensor, rewards: torch.Tensor,
               dones: torch.Tensor, gamma: float = 0.99, eps: Optional[float] = None):
    """Batched ``finish_episode`` (examples/ball_cnn_ac3.py:222-246) over a recorded rollout.

    obs (T, N, F) u8 -- the obs each action was chosen from; actions (T, N); rewards (T, N)
    f64; dones (T, N) bool.  Every maximal run of an env's steps that ends at a done (or at
    the horizon) is one episode, as ``policy.rewards`` / ``policy.saved_actions`` are in the
    reference.  Per episode, exactly as there:
      R_t = r_t + gamma R_{t+1} (python floats), then torch.tensor(R) (fp32),
      R^ = (R - R.mean()) / (R.std() + eps)          (unbiased std, eps = fp32 eps),
      policy loss  sum_t -log pi(a_t|s_t) * (R^_t - v_t.item()),
      value loss   sum_t smooth_l1(v_t, R^_t).
    Episodes of one step are skipped (the driver only trains when t > 0, :614).
    log pi and v are recomputed from ``obs`` with autograd (the rollout's own values are
    the same forward, taken without a graph).  Returns (policy_loss, value_loss) sums.
    """
    import numpy as np
    eps = float(np.finfo(np.float32).eps) if eps is None else eps
    T, N = rewards.shape
    dev = rewards.device
    d64 = dones.to(torch.float64)
    R = torch.empty(T, N, dtype=torch.float64, device=dev)
    acc = torch.zeros(N, dtype=torch.float64, device=dev)
    for t in range(T - 1, -1, -1):
        acc = rewards[t].to(torch.float64) + gamma * acc * (1.0 - d64[t])
        R[t] = acc
    R32 = R.to(torch.float32)
    # episode id of every (t, env): dones strictly before t in that env, then env
    seg = (torch.cumsum(dones.to(torch.int64), 0) - dones.to(torch.int64)) * N + torch.arange(N, device=dev)
    _, sid = torch.unique(seg.reshape(-1), return_inverse=True)
    S = int(sid.max()) + 1
    flat = R32.reshape(-1)
    cnt = torch.bincount(sid, minlength=S).to(torch.float32)
    mean = torch.zeros(S, device=dev).index_add_(0, sid, flat) / cnt
    dev2 = (flat - mean[sid]) ** 2
    var = torch.zeros(S, device=dev).index_add_(0, sid, dev2) / (cnt - 1).clamp(min=1)
    valid = (cnt > 1)[sid]
    Rn = (flat - mean[sid]) / (var.sqrt()[sid] + eps)
    probs, v = policy(obs.reshape(T * N, -1).float())
    v = v.squeeze(-1)
    logp = torch.log(probs.gather(-1, actions.reshape(-1, 1).long()).squeeze(-1))
    adv = Rn - v.detach()
    pl = -(logp * adv)[valid].sum()
    vl = torch.nn.functional.smooth_l1_loss(v[valid], Rn[valid], reduction="sum")
    return pl, vl


def a2c_update(rollout: "Rollout", optimizer, gamma: float = 0.99):
    """One A2C step on a recorded rollout (record_obs=True): loss.backward(), optimizer.step(),
    then re-pack the new weights for the HIP policy kernel.  Returns the loss value."""
    if rollout.obs is None:
        raise ValueError("a2c_update needs Rollout(record_obs=True)")
    pl, vl = a2c_losses(rollout.policy, rollout.obs[:-1], rollout.actions, rollout.rewards, rollout.dones, gamma)
    loss = pl + vl
    optimizer.zero_grad()
    loss.backward()
    optimizer.step()
    if rollout.hp is not None:
        rollout.hp.load(rollout.policy)
    return float(loss.detach())
