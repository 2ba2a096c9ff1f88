"""CPU: the Policy mirror loads the reference's trained weights (fixtures) and
torch_select_action's inverse-CDF draw behaves as Categorical sampling."""
import numpy as np
import torch

from gym_ballenv_amd.policy import HIDDEN, Policy, reference_weights, torch_select_action


def test_reference_weight_fixtures_load():
    for W in (5, 10):
        p = reference_weights(W)
        assert p is not None
        pol = Policy.from_npz(p, W)
        assert pol.fc1.in_features == 4 + W * W and pol.hidden_layer == HIDDEN[W]
        probs, v = pol(torch.zeros(3, 4 + W * W))
        assert torch.allclose(probs.sum(-1), torch.ones(3))


def test_inverse_cdf_draw_is_categorical():
    torch.manual_seed(0)
    pol = Policy.from_npz(reference_weights(10), 10)
    x = torch.zeros(1, 104)
    x[0, 1] = 1
    x = x.repeat(200000, 1)
    u = torch.rand(200000)
    with torch.no_grad():
        a, lp, v, probs = torch_select_action(pol, x, u)
    freq = torch.bincount(a, minlength=9).double() / a.numel()
    assert torch.allclose(freq, probs[0].double(), atol=4e-3)
    assert torch.allclose(lp, torch.log(probs[0, a]))


def test_policy_uniforms_oracle_range():
    from oracle import oracle
    import gym_ballenv_amd as gb
    cfg = gb.EnvConfig().to_abi(10000, 10)
    u = oracle.policy_uniforms(cfg, np.arange(10000) % 7, np.arange(10000) % 1000, 42)
    assert u.min() >= 0 and u.max() < 1 and abs(u.mean() - 0.5) < 0.01
