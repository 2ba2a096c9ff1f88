"""be_rollout (fused multi-step) == that many be_step calls, bit for bit.

The fused kernel keeps each env's state in registers for K steps; every Philox
draw is keyed by per-env state, so its per-step outputs (obs, reward, done,
truncated, final return/length), the state it leaves and the per-wave stats
slots must equal K launches of the fixed-shape step kernel exactly.  Configs
outside the fixed shape take be_rollout's be_step loop and are checked the same
way.  The step path itself is pinned to the oracle / reference golden vectors in
test_gpu_parity.py.
"""
import numpy as np
import pytest
import torch

from test_gpu_parity import KEYS, make_env, np_state

pytestmark = pytest.mark.gpu


def _run_pair(cfg_py, N, W, K, chunks, seed=7, terminal=False, lens=None, status=None):
    """Env A: K be_step calls.  Env B: be_rollout over `chunks` (step counts summing to K).  status: the
    device-status text both envs must report at the end (None: no status bit)."""
    a, b = (make_env(cfg_py, N, W, "cuda:0", seed=seed, terminal_obs=terminal) for _ in range(2))
    acts = a.sample_actions(K, seed=seed + 1)
    a.reset()
    b.reset()
    if lens is not None:   # random episode phases: goal changes and TimeLimit truncations early on
        a.ep_len.copy_(lens)
        b.ep_len.copy_(lens)
    F = 4 + W * W
    ref = {"obs": np.empty((K, N, F), np.uint8), "reward": np.empty((K, N)), "done": np.empty((K, N), bool),
           "truncated": np.empty((K, N), bool), "final_return": np.empty((K, N)), "final_len": np.empty((K, N), np.int32)}
    for t in range(K):
        obs, r, d, info = a.step(acts[t])
        ref["obs"][t], ref["reward"][t], ref["done"][t] = obs.cpu().numpy(), r.cpu().numpy(), d.cpu().numpy()
        ref["truncated"][t] = info["truncated"].cpu().numpy()
        ref["final_return"][t] = info["final_return"].cpu().numpy()
        ref["final_len"][t] = info["final_len"].cpu().numpy()
        if terminal:
            ref.setdefault("terminal_obs", np.zeros((K, N, F), np.uint8))[t] = info["terminal_obs"].cpu().numpy()
    t0 = 0
    for k in chunks:
        obs, r, d, info = b.rollout(acts[t0:t0 + k])
        sl = slice(t0, t0 + k)
        np.testing.assert_array_equal(obs.cpu().numpy(), ref["obs"][sl], err_msg=f"obs, steps {t0}..")
        np.testing.assert_array_equal(r.cpu().numpy(), ref["reward"][sl], err_msg=f"reward, steps {t0}..")
        np.testing.assert_array_equal(d.cpu().numpy(), ref["done"][sl], err_msg=f"done, steps {t0}..")
        np.testing.assert_array_equal(info["truncated"].cpu().numpy(), ref["truncated"][sl])
        dm = ref["done"][sl]   # final_* are written for done rows only
        np.testing.assert_array_equal(info["final_return"].cpu().numpy()[dm], ref["final_return"][sl][dm])
        np.testing.assert_array_equal(info["final_len"].cpu().numpy()[dm], ref["final_len"][sl][dm])
        if terminal:   # rows of envs that reset on that step
            np.testing.assert_array_equal(info["terminal_obs"].cpu().numpy()[dm], ref["terminal_obs"][sl][dm])
        t0 += k
    assert t0 == K
    sa, sb = np_state(a), np_state(b)
    for k in KEYS:
        np.testing.assert_array_equal(sb[k], sa[k], err_msg=f"final state[{k}]")
    np.testing.assert_array_equal(b.stats_buf.cpu().numpy(), a.stats_buf.cpu().numpy())
    for e in (a, b):
        if status is None:
            e.status()
        else:
            from gym_ballenv_amd._abi import BallEnvError
            with pytest.raises(BallEnvError, match=status):
                e.status()
    n_done = int(ref["done"].sum())
    a.close()
    b.close()
    return n_done


@pytest.mark.parametrize("W,N", [(10, 65536), (5, 4096), (10, 1008)])
def test_rollout_matches_steps_default(gpu, W, N):
    """Default config (fixed shape -> the fused kernel); N=1008 leaves a partial last block."""
    from gym_ballenv_amd.config import EnvConfig
    n_done = _run_pair(EnvConfig(), N, W, 60, (1, 25, 34))
    assert n_done > 0


@pytest.mark.parametrize("W", [10, 5])
def test_rollout_mass_truncation(gpu, W):
    """time_limit 20: every env of every wave resets on the same steps (multi-env reset passes);
    terminal_obs rows of the reset envs equal be_step's."""
    from gym_ballenv_amd.config import EnvConfig
    n_done = _run_pair(EnvConfig(time_limit=20), 20000, W, 45, (45,), terminal=True)
    assert n_done >= 2 * 20000


def test_rollout_generic_config(gpu):
    """A config outside the fixed shape (7 static + 3 dynamic, W=7): be_rollout loops be_step."""
    from gym_ballenv_amd.config import EnvConfig
    _run_pair(EnvConfig(num_static=7, num_dynamic=3, time_limit=30), 2048, 7, 40, (40,), terminal=True)


def test_rollout_errors(gpu):
    from gym_ballenv_amd import BallEnvError
    from gym_ballenv_amd.config import EnvConfig
    env = make_env(EnvConfig(), 1001, 5, gpu)   # 1001 * 29 is not a multiple of 16
    env.reset()
    with pytest.raises(BallEnvError, match="% 16 == 0"):
        env.rollout(torch.zeros(3, 1001, dtype=torch.uint8, device=gpu))
    with pytest.raises(ValueError):
        env.rollout(torch.zeros(3, 1000, dtype=torch.uint8, device=gpu))
    env.close()
    env = make_env(EnvConfig(), 1024, 10, gpu, obs_f32=True)
    with pytest.raises(ValueError, match="u8 obs only"):
        env.rollout(torch.zeros(3, 1024, dtype=torch.uint8, device=gpu))
    env.close()


def _policy_pair(cfg_py, N, W, T, chunk, record, policy=None, horizons=2, seed=11, status=None):
    """Rollout(backend="hip") (two launches per step) vs Rollout(backend="fused") (be_policy_rollout).
    status: the device-status text both envs must report at the end (None: no status bit)."""
    from gym_ballenv_amd.policy import Policy, reference_weights
    from gym_ballenv_amd.rollout import Rollout
    if policy is None:
        path = reference_weights(W)
        torch.manual_seed(0)
        policy = Policy.from_npz(path, W) if path else Policy(W)
    envs = [make_env(cfg_py, N, W, "cuda:0", seed=seed) for _ in range(2)]
    ros = []
    for e, be in zip(envs, ("hip", "fused")):
        e.reset()
        ros.append(Rollout(e, policy, horizon=T, backend=be, record_obs=record, seed=0x5E1EC7, chunk=chunk))
    for h in range(horizons):
        for r in ros:
            r.run_eager()
        a, b = ros
        for name in ("actions", "log_probs", "values", "rewards", "dones"):
            np.testing.assert_array_equal(getattr(b, name).cpu().numpy(), getattr(a, name).cpu().numpy(),
                                          err_msg=f"horizon {h}: {name}")
        if record:
            np.testing.assert_array_equal(b.obs.cpu().numpy(), a.obs.cpu().numpy(), err_msg=f"horizon {h}: obs")
        np.testing.assert_array_equal(envs[1].obs.cpu().numpy(), envs[0].obs.cpu().numpy(), err_msg="env.obs")
        sa, sb = np_state(envs[0]), np_state(envs[1])
        for k in KEYS:
            np.testing.assert_array_equal(sb[k], sa[k], err_msg=f"horizon {h}: state[{k}]")
        np.testing.assert_array_equal(envs[1].stats_buf.cpu().numpy(), envs[0].stats_buf.cpu().numpy())
    n_done = int(ros[0].dones.sum())
    lit = int((ros[0].obs[:, :, 4:].amax(-1) > 0).sum()) if record else -1
    for r, e in zip(ros, envs):
        if status is None:
            e.status()
        else:
            from gym_ballenv_amd._abi import BallEnvError
            with pytest.raises(BallEnvError, match=status):
                e.status()
        r.close()
        e.close()
    return n_done, lit


@pytest.mark.parametrize("W,N,record", [(10, 65536, False), (10, 65536, True), (5, 4096, True), (10, 1008, True)])
def test_policy_rollout_matches_two_launch_loop(gpu, W, N, record):
    """Fused config-5 rollout == be_policy_act + be_step per step, bit for bit (actions, log_prob,
    value, reward, done, recorded obs, env.obs, state, stats), over two horizons of 3 chunks."""
    from gym_ballenv_amd.config import EnvConfig
    n_done, lit = _policy_pair(EnvConfig(), N, W, 50, 20, record)
    assert n_done > 0
    if record:
        assert lit > 0   # some obs took the dense MFMA path


def test_policy_rollout_dense_heavy(gpu):
    """time_limit 15 and a random-init policy: many resets and many lit windows per block."""
    from gym_ballenv_amd.config import EnvConfig
    from gym_ballenv_amd.policy import Policy
    torch.manual_seed(3)
    n_done, lit = _policy_pair(EnvConfig(time_limit=15), 8192, 10, 40, 40, True, policy=Policy(10))
    assert n_done >= 2 * 8192 and lit > 0


def test_policy_rollout_generic_config(gpu):
    """An env outside the fixed shape (9 static + 4 dynamic): be_policy_rollout loops the two launches."""
    from gym_ballenv_amd.config import EnvConfig
    _policy_pair(EnvConfig(num_static=9, num_dynamic=4, time_limit=40), 2048, 10, 30, 30, True)


def test_fused_rollouts_shard_invariance(gpu):
    """Config 4's sharding through both fused modes: a global env's trajectory does not depend
    on how the env batch is split over ranks (env_offset = the shard's first global env id)."""
    from gym_ballenv_amd.config import EnvConfig
    from gym_ballenv_amd.policy import Policy, reference_weights
    from gym_ballenv_amd.rollout import Rollout
    cfg = EnvConfig(time_limit=30)
    whole = make_env(cfg, 4096, 10, gpu, seed=9)
    parts = [make_env(cfg, n, 10, gpu, seed=9, env_offset=off) for off, n in ((0, 1024), (1024, 3072))]
    acts_w = whole.sample_actions(40, seed=4)
    acts_p = [p.sample_actions(40, seed=4) for p in parts]
    np.testing.assert_array_equal(acts_w.cpu().numpy(), torch.cat(acts_p, 1).cpu().numpy())
    for e in (whole, *parts):
        e.reset()
    ow, rw, dw, _ = (x.clone() if torch.is_tensor(x) else x for x in whole.rollout(acts_w))
    res = [p.rollout(a) for p, a in zip(parts, acts_p)]
    np.testing.assert_array_equal(ow.cpu().numpy(), torch.cat([r[0] for r in res], 1).cpu().numpy())
    np.testing.assert_array_equal(rw.cpu().numpy(), torch.cat([r[1] for r in res], 1).cpu().numpy())
    np.testing.assert_array_equal(dw.cpu().numpy(), torch.cat([r[2] for r in res], 1).cpu().numpy())
    pol = Policy.from_npz(reference_weights(10), 10)
    ros = [Rollout(e, pol, horizon=30, backend="fused", seed=0x77, chunk=30) for e in (whole, *parts)]
    for r in ros:
        r.run()
    for name in ("actions", "log_probs", "values", "rewards", "dones"):
        np.testing.assert_array_equal(getattr(ros[0], name).cpu().numpy(),
                                      torch.cat([getattr(r, name) for r in ros[1:]], 1).cpu().numpy(), err_msg=name)
    for r in ros:
        r.close()
    for e in (whole, *parts):
        e.status()
        e.close()


def test_policy_rollout_crowded_multi_round(gpu):
    """An 80x80 field: most windows are lit, so blocks list more than 4 tiles (64 envs) and the
    fused kernel takes its multi-round path (chunk partials combined into LDS logits)."""
    from gym_ballenv_amd.config import EnvConfig
    from gym_ballenv_amd.policy import Policy
    cfg = EnvConfig(screen_width=80, screen_height=80, strip_goal_x=80, strip_agent_x=80, min_spawn_dist=10.0,
                    goals=[(12, 22), (23, 33), (47, 50), (60, 40), (30, 11)], time_limit=20)
    torch.manual_seed(5)
    N, T = 4096, 30
    envs = [make_env(cfg, N, 10, "cuda:0", seed=13) for _ in range(2)]
    from gym_ballenv_amd.rollout import Rollout
    pol = Policy(10)
    ros = []
    for e, be in zip(envs, ("hip", "fused")):
        e.reset()
        ros.append(Rollout(e, pol, horizon=T, backend=be, record_obs=True, seed=3, chunk=T))
    for r in ros:
        r.run_eager()
    for name in ("actions", "log_probs", "values", "rewards", "dones", "obs"):
        np.testing.assert_array_equal(getattr(ros[1], name).cpu().numpy(), getattr(ros[0], name).cpu().numpy(),
                                      err_msg=name)
    lit = (ros[0].obs[:T, :, 4:].amax(-1) > 0).reshape(T, N // 256, 256).sum(-1)
    assert int(lit.max()) > 64, int(lit.max())   # the multi-round path ran
    for r, e in zip(ros, envs):
        e.status()
        r.close()
        e.close()


@pytest.mark.parametrize("r_obs", [21, 58])
def test_w5_small_batch_kernels_non_default_radius(gpu, r_obs, monkeypatch):
    """stepw_kernel / rolloutw_kernel (W=5, eight lanes per env) at a larger collision radius
    (R = 26 / 63: wider near boxes, more lit cells and collisions) against the one-lane kernels."""
    from gym_ballenv_amd.config import EnvConfig
    cfg = EnvConfig(radius_obstacle=r_obs, time_limit=30)
    monkeypatch.setenv("BALLENV_STEP5_LPE", "1")
    monkeypatch.setenv("BALLENV_ROLLOUT5_LPE", "8")
    e = make_env(cfg, 4096, 5, gpu, seed=3)
    assert e.kernel_name("rollout") == "rolloutw_kernel<5, 13, 5, 8>" and e.kernel_name("step") == "be_kernel<5, 0, 13, 5, true>"
    e.close()
    _run_pair(cfg, 4096, 5, 40, (15, 25), terminal=True)            # rolloutw vs one-lane steps
    monkeypatch.setenv("BALLENV_STEP5_LPE", "8")
    monkeypatch.setenv("BALLENV_ROLLOUT5_LPE", "1")
    _run_pair(cfg, 4096, 5, 40, (40,), terminal=True)                # one-lane rollout vs stepw steps


@pytest.mark.parametrize("W,lpe,N", [(10, "1", 2), (10, "1", 34), (5, "8", 16), (5, "8", 48)])
def test_fused_rollouts_tiny_batches(gpu, W, lpe, N, monkeypatch):
    """The fused rollouts at the smallest batches they take -- be_rollout writes whole 16-byte obs
    words, so N * (4 + W^2) % 16 == 0: N = 2 / 16 -- and one block past them (N = 34 / 48), through
    TimeLimit resets (tl=7) and chunks that cross them, against the step path (rollout_kernel at W=10,
    rolloutw_kernel at W=5); a batch off that grid is refused, not padded."""
    from gym_ballenv_amd._abi import BallEnvError
    from gym_ballenv_amd.config import EnvConfig
    cfg = EnvConfig(time_limit=7)
    monkeypatch.setenv("BALLENV_ROLLOUT5_LPE", lpe)
    e = make_env(cfg, N, W, gpu, seed=3)
    assert e.kernel_name("rollout") == ("rollout_kernel<10, 13, 5, 0, 1, 10>" if W == 10 else "rolloutw_kernel<5, 13, 5, 8>")
    e.close()
    _run_pair(cfg, N, W, 20, (3, 9, 8), terminal=True)
    bad = make_env(cfg, N - 1, W, gpu, seed=3)
    with pytest.raises(BallEnvError, match="16-byte aligned"):
        bad.rollout(bad.sample_actions(2, seed=1))
    bad.close()


@pytest.mark.parametrize("W,lpe", [(10, "1"), (5, "8")])
def test_fused_rollouts_rejection_limit(gpu, W, lpe, monkeypatch):
    """The fused rollouts' autoreset (wave_resets in rollout_kernel / rolloutw_kernel) on the 20 x 30
    field of test_gpu_parity.py::test_reset_rejection_limit, where every reset loop stops at its
    4 096-draw bound and every env resets every step: bit for bit the step path's trajectory (and, at
    W=10, the fused policy rollout its two-launch loop's), and both report the bound."""
    from gym_ballenv_amd.config import EnvConfig
    cfg = EnvConfig(screen_width=20, screen_height=30, strip_obs_y=5, strip_goal_x=20, strip_agent_x=20, time_limit=3)
    monkeypatch.setenv("BALLENV_ROLLOUT5_LPE", lpe)
    e = make_env(cfg, 256, W, gpu, seed=3)
    assert e.kernel_name("rollout") == ("rollout_kernel<10, 13, 5, 0, 1, 10>" if W == 10 else "rolloutw_kernel<5, 13, 5, 8>")
    e.close()
    _run_pair(cfg, 256, W, 6, (2, 4), terminal=True, status="reset rejection limit")
    if W == 10:   # the config-5 fused policy rollout's autoreset (be_policy_rollout) against its two-launch loop
        n_done, _ = _policy_pair(cfg, 256, W, 6, 3, False, horizons=1, status="reset rejection limit")
        assert n_done == 256 * 6


@pytest.mark.parametrize("r_obs", [21, 58])
def test_fused_rollouts_non_default_radius(gpu, r_obs):
    """A larger collision radius R = radius_obstacle + radius_agent grows the fused kernels' LDS
    (near lists, row-span table).  At R >= 26 the config-5 kernel no longer fits the CU's 160 KB,
    so be_policy_rollout must take its two-launch fallback instead of failing the launch; the
    random-action rollout still fits at R = 63 and stays fused.  Both equal the per-step paths."""
    from gym_ballenv_amd.config import EnvConfig
    cfg = EnvConfig(radius_obstacle=r_obs, time_limit=40)
    e = make_env(cfg, 4096, 10, gpu, seed=3)
    assert e.kernel_name("rollout") == "rollout_kernel<10, 13, 5, 0, 1, 10>"
    e.close()
    _run_pair(cfg, 4096, 10, 40, (15, 25), terminal=True)
    n_done, lit = _policy_pair(cfg, 4096, 10, 30, 30, True)
    assert lit > 0


@pytest.mark.parametrize("N,tl,lpe,terminal", [(4096, 1000, "8", True), (4096, 20, "4", True), (1008, 7, "8", True),
                                              (20000, 20, "8", False)])
def test_rolloutw_matches_steps(gpu, N, tl, lpe, terminal, monkeypatch):
    """rolloutw_kernel (W=5, 8 / 4 lanes per env, 32-env blocks; the small-batch fused rollout) ==
    that many be_step calls of the one-lane step kernel, bit for bit -- per-step obs, reward, done,
    truncated, final return / length, terminal obs, the state left behind and the stats slots
    (folded every 32 steps in LDS) -- through mass truncation and partial blocks / waves, over
    chunks that cross the 32-step fold window."""
    from gym_ballenv_amd.config import EnvConfig
    monkeypatch.setenv("BALLENV_ROLLOUT5_LPE", lpe)
    monkeypatch.setenv("BALLENV_STEP5_LPE", "1")
    e = make_env(EnvConfig(time_limit=tl), N, 5, gpu, seed=3)
    assert e.kernel_name("rollout") == f"rolloutw_kernel<5, 13, 5, {lpe}>"
    assert e.kernel_name("step") == "be_kernel<5, 0, 13, 5, true>"
    e.close()
    cfg = EnvConfig(time_limit=tl)
    lens = torch.from_numpy(np.random.default_rng(N + tl).integers(0, tl, N).astype(np.int32)).to(gpu)
    n_done = _run_pair(cfg, N, 5, 75, (1, 40, 34), terminal=terminal, lens=lens)
    assert n_done > 0
