"""GPU: be_policy_act (csrc/policy.hip) vs the reference's Policy / select_action
(examples/ball_cnn_ac3.py:109-146, 210-220) run in plain PyTorch fp32 on the CPU.

Floating point, so a tolerance, written here:
* probs, value, log_prob: |hip - torch32| <= 2e-5 (abs), and the HIP error
  against an fp64 evaluation of the same weights is at most 4x torch fp32's own
  error + 1e-6 (the fixed-point fc1 is as accurate as an fp32 GEMM);
* action: identical to the inverse-CDF draw on the torch probs with the same
  Philox uniform (oracle.policy_uniforms), except where that uniform lies within
  1e-5 of a CDF boundary (counted and bounded).
"""
import numpy as np
import pytest
import torch

from oracle import oracle

pytestmark = pytest.mark.gpu

TOL = 2e-5


def make(dev, N, W, seed=0x1234, **kw):
    import gym_ballenv_amd as gb
    env = gb.BatchedBallEnv(N, W, gb.EnvConfig(), device=dev, seed=seed, **kw)
    env.reset()
    return env


def ref_policy(W, hidden=None, A=9, seed=0):
    from gym_ballenv_amd.policy import Policy, reference_weights
    if hidden is None and reference_weights(W):
        return Policy.from_npz(reference_weights(W), W)
    torch.manual_seed(seed)
    return Policy(W, hidden=hidden, num_actions=A)


def check_act(env, pol, hp, obs_dev, seed):
    from gym_ballenv_amd.policy import torch_select_action
    a, lp, v, pr = hp.act(obs_dev, seed=seed)
    a, lp, v, pr = (x.cpu() for x in (a, lp, v, pr))
    cfg = env._abi_cfg
    ep = env.episode.cpu().numpy().view(np.uint32)
    u = torch.from_numpy(oracle.policy_uniforms(cfg, ep, env.ep_len.cpu().numpy(), seed))
    obs = obs_dev.cpu()
    with torch.no_grad():
        ra, rlp, rv, rpr = torch_select_action(pol.float(), obs, u)
        p64 = pol.double()
        pr64, v64 = p64(obs.double())
        pol.float()
    err_hip = (pr.double() - pr64).abs().max().item()
    err_t32 = (rpr.double() - pr64).abs().max().item()
    assert (pr - rpr).abs().max().item() <= TOL
    assert (v - rv).abs().max().item() <= TOL
    assert err_hip <= 4 * err_t32 + 1e-6, (err_hip, err_t32)
    assert (v.double() - v64.squeeze(-1)).abs().max().item() <= 4 * (rv.double() - v64.squeeze(-1)).abs().max().item() + 1e-6
    cdf = rpr.cumsum(-1)
    near = ((cdf - u.unsqueeze(-1)).abs() < 1e-5).any(-1)
    mism = a.long() != ra
    assert not (mism & ~near).any(), f"{int((mism & ~near).sum())} action mismatches away from CDF boundaries"
    assert int(near.sum()) <= max(4, obs.shape[0] // 1000)
    ok = ~mism
    assert (lp[ok] - rlp[ok]).abs().max().item() <= TOL
    return a


@pytest.mark.parametrize("W", [10, 5])
def test_policy_reference_weights_env_obs(gpu, W):
    """The reference's trained Policy(W) on obs the step kernel produced, along a random rollout."""
    from gym_ballenv_amd.policy import HipPolicy
    env = make(gpu, 4096, W)
    pol = ref_policy(W)
    hp = HipPolicy(env, pol, probs=True)
    acts = env.sample_actions(40, seed=9)
    lit = 0
    for t in range(40):
        env.step(acts[t])
        if t % 8 == 7:
            check_act(env, pol, hp, env.obs, seed=77 + t)
            lit += int((env.obs[:, 4:].sum(1) > 0).sum())
    assert lit > 0          # some windows saw obstacles
    hp.close(); env.close()


@pytest.mark.parametrize("W,hidden,A,N", [(10, 208, 9, 1000), (10, 100, 5, 333), (7, 256, 15, 130), (3, 16, 1, 70)])
def test_policy_random_weights_and_obs(gpu, W, hidden, A, N):
    """Random weights (generic and ragged shapes, N not a multiple of 64) on random 0/1 obs, incl. all-ones rows."""
    from gym_ballenv_amd.policy import HipPolicy
    env = make(gpu, N, W)
    pol = ref_policy(W, hidden=hidden, A=A, seed=W * 1000 + hidden)
    with torch.no_grad():
        for prm in pol.parameters():
            prm.mul_(3.0)        # wider logits than init
    hp = HipPolicy(env, pol, probs=True)
    g = torch.Generator().manual_seed(N)
    obs = (torch.rand(N, env.obs_dim, generator=g) < 0.5).to(torch.uint8)
    obs[: N // 10] = 1
    obs[N // 10: N // 5] = 0
    check_act(env, pol, hp, obs.to(gpu).contiguous(), seed=5)
    hp.close(); env.close()


def test_policy_reload_and_determinism(gpu):
    """Same state + seed -> same draws; be_policy_load re-packs new weights."""
    from gym_ballenv_amd.policy import HipPolicy
    env = make(gpu, 2048, 10)
    pol = ref_policy(10)
    hp = HipPolicy(env, pol, probs=True)
    a1 = hp.act(seed=3)[0].clone()
    a2 = hp.act(seed=3)[0].clone()
    assert torch.equal(a1, a2)
    a3 = hp.act(seed=4)[0].clone()
    assert not torch.equal(a1, a3)
    pol2 = ref_policy(10, hidden=208, seed=11)
    hp.load(pol2)
    check_act(env, pol2, hp, env.obs, seed=3)
    hp.close(); env.close()


def test_rollout_hip_graph_matches_eager(gpu):
    """A captured T-step rollout (policy + step per step, one graph) == the same steps run eagerly."""
    from gym_ballenv_amd import Rollout
    pol = ref_policy(10)
    outs = []
    for mode in ("eager", "graph"):
        env = make(gpu, 1024, 10, seed=21)
        ro = Rollout(env, pol, horizon=64, backend="hip", seed=99)
        if mode == "eager":
            ro.run_eager()
        else:
            ro.capture(chunk=32)
            ro.run()
        torch.cuda.synchronize()
        outs.append([x.cpu().clone() for x in (ro.actions, ro.log_probs, ro.values, ro.rewards, ro.dones)] +
                    [env.obs.cpu().clone()])
        env.status()
        ro.close(); env.close()
    for x, y in zip(*outs):
        assert torch.equal(x, y)


def test_rollout_recorded_obs_replays_through_torch(gpu):
    """record_obs: every recorded obs row reproduces the recorded log_prob/value in torch fp32
    (what an A2C update recomputes), and the recorded rewards/dones match an env stepped with the same actions."""
    from gym_ballenv_amd import Rollout
    from gym_ballenv_amd.policy import torch_select_action
    pol = ref_policy(10)
    env = make(gpu, 512, 10, seed=5)
    ro = Rollout(env, pol, horizon=20, backend="hip", record_obs=True, seed=1)
    ro.run_eager()
    torch.cuda.synchronize()
    with torch.no_grad():
        for t in range(20):
            probs, v = pol(ro.obs[t].cpu().float())
            lp = torch.log(probs.gather(-1, ro.actions[t].cpu().long().unsqueeze(-1))).squeeze(-1)
            assert (lp - ro.log_probs[t].cpu()).abs().max().item() <= TOL
            assert (v.squeeze(-1) - ro.values[t].cpu()).abs().max().item() <= TOL
    env2 = make(gpu, 512, 10, seed=5)
    for t in range(20):
        obs, r, d, _ = env2.step(ro.actions[t])
        assert torch.equal(obs, ro.obs[t + 1])
        assert torch.equal(r, ro.rewards[t]) and torch.equal(d, ro.dones[t])
    R = ro.discounted_returns(0.9)
    r, d = ro.rewards.cpu(), ro.dones.cpu()
    acc = torch.zeros(512, dtype=torch.float64)
    for t in range(19, -1, -1):
        acc = r[t] + 0.9 * acc * (~d[t]).double()
        assert torch.allclose(R[t].cpu(), acc)
    ro.close(); env.close(); env2.close()


def test_rollout_torch_backend_runs(gpu):
    from gym_ballenv_amd import Rollout
    pol = ref_policy(10)
    env = make(gpu, 1024, 10)
    ro = Rollout(env, pol, horizon=16, backend="torch")
    ro.capture(chunk=16)
    ro.run()
    torch.cuda.synchronize()
    assert int(ro.actions.max()) < 9
    env.status()
    ro.close(); env.close()


def test_a2c_update_on_gpu_rollout(gpu):
    """rollout (HIP) -> a2c_update (torch autograd on the recorded obs) -> re-pack: the loss is
    finite, the weights move, and the HIP kernel then acts with the new weights."""
    import copy
    from gym_ballenv_amd import Rollout, a2c_update
    from gym_ballenv_amd.policy import Policy, reference_weights
    pol = Policy.from_npz(reference_weights(10), 10).to(gpu)
    w0 = copy.deepcopy(pol.state_dict())
    env = make(gpu, 512, 10, seed=3)
    ro = Rollout(env, pol, horizon=32, backend="hip", record_obs=True, seed=2)
    ro.run_eager()
    opt = torch.optim.Adam(pol.parameters(), lr=1e-2)
    loss = a2c_update(ro, opt, gamma=0.99)
    assert np.isfinite(loss)
    assert not torch.equal(w0["fc1.weight"], pol.fc1.weight.detach())
    from gym_ballenv_amd.policy import HipPolicy
    hp2 = HipPolicy(env, pol, probs=True)
    a_new = check_act(env, pol.cpu(), hp2, env.obs, seed=9)
    assert torch.equal(ro.hp.act(seed=9)[0].cpu(), a_new)      # the rollout's kernel was re-packed
    hp2.close(); ro.close(); env.close()


@pytest.mark.parametrize("W", [10, 5])
def test_policy_sparse_path_equals_dense(gpu, W, monkeypatch):
    """The empty-window fast path (table of the 4 quadrant-only obs + compacted lit envs) is
    bit-identical to running every env through the matrix cores (BALLENV_POLICY_DEBUG=32)."""
    from gym_ballenv_amd.policy import HipPolicy
    env = make(gpu, 3000, W, seed=8)
    acts = env.sample_actions(30, seed=4)
    for t in range(30):
        env.step(acts[t])
    pol = ref_policy(W)
    g = torch.Generator().manual_seed(1)
    rand_obs = (torch.rand(3000, env.obs_dim, generator=g) < 0.05).to(torch.uint8)
    rand_obs[:, :4] = 0
    rand_obs[torch.arange(3000), torch.randint(0, 4, (3000,), generator=g)] = 1
    hps = []
    for dbg in ("0", "32"):
        monkeypatch.setenv("BALLENV_POLICY_DEBUG", dbg)
        hps.append(HipPolicy(env, pol, probs=True))
    monkeypatch.delenv("BALLENV_POLICY_DEBUG")
    lit = int((env.obs[:, 4:].sum(1) > 0).sum())
    assert 0 < lit < 3000
    for obs in (env.obs, rand_obs.to(gpu)):
        r = [[x.clone() for x in hp.act(obs, seed=6)] for hp in hps]
        for a, b in zip(*r):
            assert torch.equal(a, b)
    for hp in hps:
        hp.close()
    env.close()
