"""GPU (HIP, gfx950) parity: libballenv.so vs the reference's golden vectors and
vs the C oracle.  Bar: bit-exact everywhere (rewards compared with ==, obs /
done / state bit for bit); only the f64 stats sums (atomic-order dependent) get
a tolerance.
"""
import numpy as np
import pytest
import torch

from helpers import env_config, init_state, load, step_tape, window_config, window_state
from oracle import oracle

pytestmark = pytest.mark.gpu

KEYS = ("agent", "goal", "prev_dist", "total_dist", "ep_return", "ep_len", "episode", "static_obs", "dyn_obs",
        "dyn_goal")


def make_env(cfg_py, n, W, dev, seed=0xBA11, env_offset=0, **kw):
    from gym_ballenv_amd import BatchedBallEnv
    return BatchedBallEnv(n, W, cfg_py, device=dev, seed=seed, env_offset=env_offset, **kw)


def load_np_state(env, st):
    env.load_state_dict({k: torch.from_numpy(np.ascontiguousarray(st[k])) for k in KEYS})


def np_state(env):
    d = {k: getattr(env, k).cpu().numpy().copy() for k in KEYS}
    d["episode"] = d["episode"].view(np.uint32)
    return d


def assert_state_equal(env, st, msg=""):
    got = np_state(env)
    for k in KEYS:
        np.testing.assert_array_equal(got[k], st[k], err_msg=f"{msg} state[{k}]")


@pytest.mark.parametrize("name,windows", [("rollouts_default", (5, 10)), ("rollouts_directed", (5, 10)),
                                          ("rollouts_custom", (7,))])
def test_golden_rollouts(gpu, name, windows):
    fx = load(name)
    cfg_py = env_config(fx["config"])
    E, T = fx["actions"].shape
    for W in windows:
        env = make_env(cfg_py, E, W, gpu, obs_f32=False)
        load_np_state(env, init_state(fx))
        np.testing.assert_array_equal(env.observe().cpu().numpy(), fx[f"init_obs{W}"])
        acts = torch.from_numpy(fx["actions"]).to(gpu)
        for t in range(T):
            tape = torch.from_numpy(step_tape(fx, t)).to(gpu) if cfg_py.num_dynamic else None
            obs, reward, done, info = env.step(acts[:, t].contiguous(), draw_tape=tape)
            np.testing.assert_array_equal(reward.cpu().numpy(), fx["reward"][:, t], err_msg=f"W={W} t={t}")
            np.testing.assert_array_equal(done.cpu().numpy(), fx["done"][:, t].astype(bool), err_msg=f"t={t}")
            np.testing.assert_array_equal(obs.cpu().numpy(), fx[f"obs{W}"][:, t], err_msg=f"W={W} t={t}")
            np.testing.assert_array_equal(env.agent.cpu().numpy(), fx["agent"][:, t])
            if cfg_py.num_dynamic:
                np.testing.assert_array_equal(env.dyn_obs.cpu().numpy().transpose(1, 0, 2), fx["dyn"][:, t])
                np.testing.assert_array_equal(env.dyn_goal.cpu().numpy().T, fx["dyn_goal"][:, t])
            np.testing.assert_array_equal(env.ep_return.cpu().numpy(), fx["ep_return"][:, t])
        env.status()
        env.close()


def test_golden_crafted(gpu):
    fx = load("crafted")
    cfg_py = env_config(fx["config"])
    E = fx["actions"].shape[0]
    for W in (5, 10):
        env = make_env(cfg_py, E, W, gpu)
        load_np_state(env, init_state(fx))
        tape = torch.from_numpy(np.ascontiguousarray(fx["tape"].transpose(1, 2, 0).astype(np.int16))).to(gpu)
        obs, reward, done, _ = env.step(torch.from_numpy(fx["actions"]).to(gpu), draw_tape=tape)
        r, d, o = reward.cpu().numpy(), done.cpu().numpy(), obs.cpu().numpy()
        for e, nm in enumerate(fx["names"]):
            assert r[e] == fx["reward"][e], nm
            assert d[e] == bool(fx["done"][e]), nm
            assert np.array_equal(o[e], fx[f"obs{W}"][e]), nm
        np.testing.assert_array_equal(env.dyn_obs.cpu().numpy().transpose(1, 0, 2), fx["dyn"])
        np.testing.assert_array_equal(env.dyn_goal.cpu().numpy().T, fx["dyn_goal"])
        env.close()


@pytest.mark.parametrize("which", ["default", "custom"])
def test_golden_resets(gpu, which):
    fx = load("resets")
    g = {k[len(which) + 1:]: v for k, v in fx.items() if k.startswith(which + "_")}
    cfg_py = env_config(g["config"])
    E = g["seeds"].shape[0]
    env = make_env(cfg_py, E, 5, gpu)
    tape = torch.from_numpy(np.ascontiguousarray(g["tape"].T.astype(np.int16))).to(gpu)
    env.reset(reset_tape=tape)
    env.status()
    st = np_state(env)
    np.testing.assert_array_equal(st["agent"], g["agent"])
    np.testing.assert_array_equal(st["goal"], g["goal"])
    np.testing.assert_array_equal(st["prev_dist"], g["prev_dist"])
    np.testing.assert_array_equal(st["total_dist"], g["total_dist"])
    np.testing.assert_array_equal(st["static_obs"][:cfg_py.num_static].transpose(1, 0, 2), g["static"])
    np.testing.assert_array_equal(st["dyn_obs"][:cfg_py.num_dynamic].transpose(1, 0, 2), g["dyn"])
    np.testing.assert_array_equal(st["dyn_goal"][:cfg_py.num_dynamic].T, g["dyn_goal"])
    env.close()


@pytest.mark.parametrize("name", ["windows", "windows_custom"])
def test_golden_windows(gpu, name):
    fx = load(name)
    for W in fx["windows"]:
        W = int(W)
        st, K = window_state(fx[f"W{W}_agent"], fx[f"W{W}_goal"], fx[f"W{W}_obst"], fx[f"W{W}_nobs"])
        cfg_py = window_config(fx["env"], K)
        n = st["agent"].shape[0]
        env = make_env(cfg_py, n, W, gpu, obs_f32=True)
        load_np_state(env, st)
        obs = env.observe().cpu().numpy()
        np.testing.assert_array_equal(obs, fx[f"W{W}_obs"].astype(np.float32), err_msg=f"W={W}")
        np.testing.assert_array_equal(env.obs.cpu().numpy(), fx[f"W{W}_obs"], err_msg=f"W={W} u8")
        env.close()


def random_state(cfg, rng, near=True):
    """Random SoA state with obstacles clustered around agents (exercises windows + collisions)."""
    N = cfg.num_envs
    st = oracle.new_state(cfg)
    ax, ay = rng.integers(0, 501, N), rng.integers(0, 501, N)
    st["agent"][:, 0], st["agent"][:, 1] = ax, ay
    st["goal"][:, 0], st["goal"][:, 1] = rng.integers(0, 500, N), rng.integers(0, 500, N)
    st["prev_dist"][:] = rng.uniform(1, 700, N)
    st["total_dist"][:] = rng.uniform(400, 800, N)
    st["ep_len"][:] = rng.integers(0, 400, N)
    span = 30 + cfg.window
    for key, K in (("static_obs", cfg.num_static), ("dyn_obs", cfg.num_dynamic)):
        for k in range(K):
            st[key][k, :, 0] = ax + rng.integers(-span, span + 1, N)
            st[key][k, :, 1] = ay + rng.integers(-span, span + 1, N)
    if cfg.num_dynamic:
        st["dyn_goal"][:cfg.num_dynamic] = rng.integers(0, cfg.num_goals, (cfg.num_dynamic, N))
    return st


def random_tape(cfg, st, rng):
    """(Nd, 2, N) draw tape whose values lie in the randint range of the branch each
    obstacle takes this step (as a recorded reference tape would)."""
    nd, N = cfg.num_dynamic, cfg.num_envs
    t = np.full((nd, 2, N), -1, np.int16)
    goals = np.array([[cfg.goals[g][0], cfg.goals[g][1]] for g in range(cfg.num_goals)])
    change = (st["ep_len"] % (cfg.goal_change_step + 1)) >= cfg.goal_change_step
    for k in range(nd):
        g = goals[st["dyn_goal"][k].astype(int)]
        tx = g[:, 0] - st["dyn_obs"][k, :, 0].astype(int)
        ty = g[:, 1] - st["dyn_obs"][k, :, 1].astype(int)
        two = (tx != 0) & (ty != 0)
        n_other = np.array([sum(1 for q in range(cfg.num_goals) if tuple(goals[q]) != tuple(goals[gi]))
                            for gi in st["dyn_goal"][k].astype(int)])
        t[k, 0] = np.where(change, rng.integers(0, 1 << 30, N) % np.maximum(n_other, 1),
                           np.where(two, rng.integers(0, 100, N), rng.integers(0, 9, N)))
        t[k, 1] = rng.integers(0, 9, N)
    return t


@pytest.mark.parametrize("W", [1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 21, 33, 64])
def test_vs_oracle_random_tape(gpu, W):
    """Tape mode on random clustered states, N not a multiple of the block size."""
    from gym_ballenv_amd.config import EnvConfig
    rng = np.random.default_rng(W)
    cfg_py = EnvConfig(autoreset=False, time_limit=0, goal_change_step=5)
    N = 3001 if W <= 21 else 515
    cfg = cfg_py.to_abi(N, W)
    st = random_state(cfg, rng)
    env = make_env(cfg_py, N, W, gpu, obs_f32=True)
    load_np_state(env, st)
    out = oracle.new_out(cfg, f32=True)
    for t in range(6):
        acts = rng.integers(0, 9, N).astype(np.uint8)
        tape = random_tape(cfg, st, rng)
        assert oracle.step(cfg, st, out, actions=acts, tape=tape) == 0
        obs, reward, done, _ = env.step(torch.from_numpy(acts).to(gpu), draw_tape=torch.from_numpy(tape).to(gpu))
        np.testing.assert_array_equal(reward.cpu().numpy(), out["reward"], err_msg=f"W={W} t={t}")
        np.testing.assert_array_equal(done.cpu().numpy(), out["done"].astype(bool))
        np.testing.assert_array_equal(obs.cpu().numpy(), out["obs"], err_msg=f"W={W} t={t}")
        np.testing.assert_array_equal(env.obs_f32.cpu().numpy(), out["obs_f32"])
        assert_state_equal(env, st, f"W={W} t={t}")
    env.status()
    env.close()


@pytest.mark.parametrize("W,N,given", [(10, 65536, False), (5, 4096, False), (10, 1000, False), (7, 333, False),
                                       (10, 65536, True), (5, 4096, True), (10, 1000, True), (7, 333, True)])
def test_vs_oracle_philox_autoreset(gpu, W, N, given):
    """Perf mode (Philox draws, in-kernel autoreset + time limit) is bit-exact against the
    oracle run with the same counters, incl. terminal obs.  given=False: in-kernel sampled
    actions (generic kernel); given=True: caller actions (the fixed-shape 13+5 kernel at
    W 5 / 10, with the wave-cooperative resets)."""
    from gym_ballenv_amd.config import EnvConfig
    cfg_py = EnvConfig(autoreset=True, time_limit=37)
    cfg = cfg_py.to_abi(N, W, seed=77)
    env = make_env(cfg_py, N, W, gpu, seed=77, terminal_obs=True)
    st = oracle.new_state(cfg)
    out = oracle.new_out(cfg, terminal=True)
    oracle.reset(cfg, st, out)
    np.testing.assert_array_equal(env.reset().cpu().numpy(), out["obs"])
    assert_state_equal(env, st, "reset")
    steps = 60 if N <= 4096 else 12
    acts = env.sample_actions(steps, seed=5) if given else None
    for t in range(steps):
        out["terminal_obs"][:] = 0
        env.terminal_obs.zero_()
        if given:
            oracle.step(cfg, st, out, actions=acts[t].cpu().numpy())
            obs, reward, done, info = env.step(acts[t])
        else:
            oracle.step(cfg, st, out)
            obs, reward, done, info = env.step()
        d = done.cpu().numpy()
        np.testing.assert_array_equal(reward.cpu().numpy(), out["reward"], err_msg=f"t={t}")
        np.testing.assert_array_equal(d, out["done"].astype(bool), err_msg=f"t={t}")
        np.testing.assert_array_equal(info["truncated"].cpu().numpy(), out["truncated"].astype(bool))
        np.testing.assert_array_equal(obs.cpu().numpy(), out["obs"], err_msg=f"t={t}")
        np.testing.assert_array_equal(info["final_return"].cpu().numpy()[d], out["final_return"][d.astype(bool)])
        np.testing.assert_array_equal(info["final_len"].cpu().numpy()[d], out["final_len"][d.astype(bool)])
        np.testing.assert_array_equal(info["terminal_obs"].cpu().numpy(), out["terminal_obs"])
        assert_state_equal(env, st, f"t={t}")
    s_gpu = env.stats_record().cpu().numpy()
    s_orc = out["stats"]
    assert s_gpu[0] == s_orc[0] and s_gpu[4] == s_orc[4] and s_gpu[5] == s_orc[5] and s_gpu[3] == s_orc[3]
    np.testing.assert_allclose(s_gpu[1:3], s_orc[1:3], rtol=1e-12, atol=1e-9)
    env.status()
    env.close()


@pytest.mark.parametrize("W", [10, 5])
def test_fixed_vs_generic_kernel(gpu, W, monkeypatch):
    """The fixed-shape step kernel (13+5 obstacles, caller actions) equals the generic one bit
    for bit, through mass truncation (every lane of every wave resets on the same step) and the
    reward/done/terminal outputs; BALLENV_GENERIC_KERNELS=1 forces the generic kernel."""
    from gym_ballenv_amd.config import EnvConfig
    cfg_py = EnvConfig(time_limit=20)
    N = 20000
    envs = []
    for generic in ("0", "1"):
        monkeypatch.setenv("BALLENV_GENERIC_KERNELS", generic)
        envs.append(make_env(cfg_py, N, W, gpu, seed=21, terminal_obs=True))
    monkeypatch.delenv("BALLENV_GENERIC_KERNELS")
    acts = envs[0].sample_actions(45, seed=8)
    for e in envs:
        e.reset()
    for t in range(45):
        res = [e.step(acts[t]) for e in envs]
        for a, b in zip(res[0][:3], res[1][:3]):
            np.testing.assert_array_equal(a.cpu().numpy(), b.cpu().numpy(), err_msg=f"t={t}")
        np.testing.assert_array_equal(res[0][3]["terminal_obs"].cpu().numpy(), res[1][3]["terminal_obs"].cpu().numpy())
        s0, s1 = np_state(envs[0]), np_state(envs[1])
        for k in KEYS:
            np.testing.assert_array_equal(s0[k], s1[k], err_msg=f"t={t} {k}")
    assert res[0][2].any()
    for e in envs:
        e.status()
        e.close()


def test_shard_invariance(gpu):
    """A global env's trajectory does not depend on how the batch is split (multi-GPU)."""
    from gym_ballenv_amd.config import EnvConfig
    cfg_py = EnvConfig(time_limit=25)
    whole = make_env(cfg_py, 1000, 10, gpu, seed=5)
    parts = [make_env(cfg_py, n, 10, gpu, seed=5, env_offset=off) for off, n in ((0, 300), (300, 700))]
    whole.reset()
    for p in parts:
        p.reset()
    for _ in range(40):
        ow, rw, dw, _ = whole.step()
        res = [p.step() for p in parts]
        np.testing.assert_array_equal(ow.cpu().numpy(), torch.cat([r[0] for r in res]).cpu().numpy())
        np.testing.assert_array_equal(rw.cpu().numpy(), torch.cat([r[1] for r in res]).cpu().numpy())
    acts_w = whole.sample_actions(8, seed=3).cpu().numpy()
    acts_p = np.concatenate([p.sample_actions(8, seed=3).cpu().numpy() for p in parts], axis=1)
    np.testing.assert_array_equal(acts_w, acts_p)
    cfg = cfg_py.to_abi(1000, 10)
    np.testing.assert_array_equal(acts_w, oracle.sample_actions(cfg, 8, 3))


def test_distance_sqrt_exhaustive(gpu):
    """Every reachable agent-goal offset (|dx|,|dy| <= 500): reward = -dist bit-exact vs numpy sqrt."""
    from gym_ballenv_amd.config import EnvConfig
    xs, ys = np.meshgrid(np.arange(501), np.arange(501), indexing="ij")
    N = xs.size
    cfg_py = EnvConfig(num_static=0, num_dynamic=0, obstacle_speed=[], goals=[], autoreset=False,
                       time_limit=0, threshold_goal=-1.0)
    env = make_env(cfg_py, N, 3, gpu)
    st = {"agent": np.stack([xs.ravel(), ys.ravel()], 1).astype(np.int16),
          "goal": np.zeros((N, 2), np.int16), "prev_dist": np.zeros(N), "total_dist": np.ones(N),
          "ep_return": np.zeros(N), "ep_len": np.zeros(N, np.int32), "episode": np.zeros(N, np.uint32),
          "static_obs": np.zeros((1, N, 2), np.int16), "dyn_obs": np.zeros((1, N, 2), np.int16),
          "dyn_goal": np.zeros((1, N), np.uint8)}
    load_np_state(env, st)
    _, reward, _, _ = env.step(torch.full((N,), 5, dtype=torch.uint8, device=gpu))   # (0, 0) move
    want = -np.sqrt((xs.ravel().astype(np.float64) ** 2 + ys.ravel().astype(np.float64) ** 2))
    np.testing.assert_array_equal(reward.cpu().numpy(), want)
    env.close()


@pytest.mark.parametrize("W", [10, 5])
def test_goal_threshold_boundaries(gpu, W):
    """done's goal test (dist < threshold_goal, ballenv_env.py:200-229) on the fixed-shape step kernels:
    every offset |dx|, |dy| <= 60 against numpy's sqrt(d2) < threshold, at thresholds on and one ulp
    either side of exact square roots (an integer d2 < n form of the test must match this too)."""
    from gym_ballenv_amd.config import EnvConfig
    r = np.arange(-60, 61)
    dx, dy = [a.ravel() for a in np.meshgrid(r, r, indexing="ij")]
    N = dx.size
    d = np.sqrt((dx.astype(np.float64) ** 2 + dy.astype(np.float64) ** 2))
    s1800 = float(np.sqrt(1800.0))
    for thr in (10.0, np.nextafter(10.0, 0.0), np.nextafter(10.0, 20.0), s1800, np.nextafter(s1800, 0.0),
                np.nextafter(s1800, 99.0), 7.5, 0.0, -1.0, 1e9):
        cfg_py = EnvConfig(autoreset=False, time_limit=0, threshold_goal=float(thr))
        env = make_env(cfg_py, N, W, gpu)   # (no autoreset: no pool, the plain fixed-shape variants)
        assert env.kernel_name("step") in ("step2_kernel<10, 13, 5, false>", "stepw_kernel<5, 13, 5, 8, false>", f"be_kernel<{W}, 0, 13, 5, false>")
        st = np_state(env)
        st["goal"][:] = (250, 250)
        st["agent"] = np.stack([250 + dx, 250 + dy], 1).astype(np.int16)
        st["static_obs"][:] = (470, 30)      # far from every agent: no collision, nothing near
        st["dyn_obs"][:] = (30, 470)
        load_np_state(env, st)
        _, _, done, _ = env.step(torch.full((N,), 5, dtype=torch.uint8, device=gpu))   # the (0, 0) move
        np.testing.assert_array_equal(done.cpu().numpy(), d < thr, err_msg=f"threshold {thr!r}")
        env.close()


@pytest.mark.parametrize("W", [10, 5])
def test_reset_rejection_limit(gpu, W):
    """A 20 x 30 field where no spawn passes the reset's rejection tests: every static obstacle overlaps
    the agent's or the goal's rectangle (ballenv_env.py:131-149, :193-197) and no goal is 50 px from
    the agent (:121-126), so every loop stops at its 4 096-draw bound.  be_reset (the block-cooperative
    reset) and the fixed-shape step kernels' autoreset (wave_resets; a collision every step) leave the
    oracle's state bit for bit -- the same last draws -- and status() reports the bound."""
    from gym_ballenv_amd._abi import BallEnvError
    from gym_ballenv_amd.config import EnvConfig
    N, T, seed = 200, 4, 5
    cfg_py = EnvConfig(screen_width=20, screen_height=30, strip_obs_y=5, strip_goal_x=20, strip_agent_x=20,
                       time_limit=3)
    env = make_env(cfg_py, N, W, gpu, seed=seed)
    assert env.kernel_name("step") in ("step2_kernel<10, 13, 5, true>", "stepw_kernel<5, 13, 5, 8, true>", f"be_kernel<{W}, 0, 13, 5, true>")
    cfg = cfg_py.to_abi(N, W, seed=seed)
    st, out = oracle.new_state(cfg), oracle.new_out(cfg)
    env.reset()
    assert oracle.reset(cfg, st, out) & 2
    with pytest.raises(BallEnvError, match="reset rejection limit"):
        env.status()
    assert_state_equal(env, st, "reset")
    acts = env.sample_actions(T, seed=seed)
    resets = 0
    for t in range(T):
        obs, reward, done, _ = env.step(acts[t])
        status = oracle.step(cfg, st, out, actions=acts[t].cpu().numpy())
        np.testing.assert_array_equal(obs.cpu().numpy(), out["obs"], err_msg=f"t={t} obs")
        np.testing.assert_array_equal(reward.cpu().numpy(), out["reward"], err_msg=f"t={t} reward")
        np.testing.assert_array_equal(done.cpu().numpy(), out["done"], err_msg=f"t={t} done")
        assert_state_equal(env, st, f"t={t}")
        resets += int(out["done"].sum())
        assert bool(status & 2) == bool(out["done"].any())   # every reset here hits the bound
        if status & 2:
            with pytest.raises(BallEnvError, match="reset rejection limit"):
                env.status()
        else:
            env.status()
    assert resets >= N   # (the TimeLimit alone ends every episode by step 3)
    env.close()


def test_large_batch_subset_vs_oracle(gpu):
    """2^20 envs (past the Infinity Cache): a contiguous slice matches the oracle run
    on just that slice (Philox streams are keyed by global env id)."""
    from gym_ballenv_amd.config import EnvConfig
    N, W, a, k = 1 << 20, 10, 700_000, 2048
    cfg_py = EnvConfig(time_limit=9)
    env = make_env(cfg_py, N, W, gpu, seed=11)
    env.reset()
    cfg = cfg_py.to_abi(k, W, env_offset=a, seed=11)
    st = oracle.new_state(cfg)
    out = oracle.new_out(cfg)
    oracle.reset(cfg, st, out)
    for t in range(12):
        obs, reward, done, _ = env.step()
        oracle.step(cfg, st, out)
        np.testing.assert_array_equal(obs[a:a + k].cpu().numpy(), out["obs"])
        np.testing.assert_array_equal(reward[a:a + k].cpu().numpy(), out["reward"])
    # global invariants on the whole batch
    o = obs.cpu().numpy()
    assert (o[:, :4].sum(1) == 1).all() and set(np.unique(o)) <= {0, 1}
    assert np.isfinite(reward.cpu().numpy()).all()
    assert (env.ep_len.cpu().numpy() < 9).all()
    env.status()
    env.close()


def test_obs_window_mask_reset(gpu):
    """Masked reset leaves other envs untouched; observe() is idempotent."""
    from gym_ballenv_amd.config import EnvConfig
    env = make_env(EnvConfig(), 777, 10, gpu, seed=1)
    env.reset()
    for _ in range(5):
        env.step()
    before = np_state(env)
    mask = torch.zeros(777, dtype=torch.bool)
    mask[::3] = True
    env.reset(mask=mask)
    after = np_state(env)
    keep = ~mask.numpy()
    for k in ("agent", "goal", "prev_dist", "ep_len"):
        np.testing.assert_array_equal(after[k][keep], before[k][keep])
    assert (after["ep_len"][mask.numpy()] == 0).all()
    o1 = env.observe().clone()
    o2 = env.observe()
    assert torch.equal(o1, o2)
    env.close()


def test_status_errors(gpu):
    from gym_ballenv_amd import BallEnvError
    from gym_ballenv_amd.config import EnvConfig
    env = make_env(EnvConfig(autoreset=False), 64, 5, gpu)
    env.reset()
    env.step(torch.full((64,), 12, dtype=torch.uint8, device=gpu))   # index >= 9
    with pytest.raises(BallEnvError, match="action index"):
        env.status()
    env.status()  # cleared
    with pytest.raises(BallEnvError, match="exhausted"):
        env.reset(reset_tape=torch.zeros(3, 64, dtype=torch.int16))
        env.status()
    env.close()


def test_compat_single_env(gpu):
    import gym_ballenv_amd as gb
    env = gb.make("gymball-v0", window=5)
    s = env.reset()
    assert len(s) == 3 + 13 + 5
    s2, r, d, info = env.step((1, 1))
    assert isinstance(r, float) and isinstance(d, bool)
    ob = env.unwrapped.window_obs(5)
    assert ob.shape == (1, 29) and ob.dtype == torch.float32 and float(ob[0, :4].sum()) == 1.0
    assert env.unwrapped.radius_rand_person == 20 and env.action_space.n == 9
    img = env.render(mode="rgb_array")
    assert img.shape == (500, 500, 3) and img.dtype == np.uint8   # the reference's 500x500 viewer
    for _ in range(1100):
        _, _, d, _ = env.step((0, 0))
        if d:
            break
    assert d  # TimeLimit(1000) or a collision


@pytest.mark.gpu
def test_save_load_state_blob_round_trip(gpu):
    """be_save_state / be_load_state (C ABI): a blob saved mid-episode, on the device
    and in host memory, restores every env bit for bit -- the next steps reproduce the same obs,
    rewards, dones and state (Philox positions included); a blob of another shape is refused."""
    from gym_ballenv_amd import BallEnvError
    from gym_ballenv_amd.config import EnvConfig
    N, W = 3000, 10
    env = make_env(EnvConfig(time_limit=25), N, W, gpu, seed=21)
    env.reset()
    acts = env.sample_actions(60, seed=5)
    for t in range(20):
        env.step(acts[t])
    dev_blob, host_blob = env.save_state(), env.save_state("cpu")
    torch.cuda.synchronize()
    assert dev_blob.numel() == host_blob.numel() and bytes(host_blob[:8].numpy()) == b"BALLENV1"
    ref = []
    for t in range(20, 60):
        obs, r, d, _ = env.step(acts[t])
        ref.append((obs.cpu().numpy(), r.cpu().numpy(), d.cpu().numpy()))
    end = np_state(env)
    for blob in (dev_blob, host_blob):
        env.load_state(blob)
        for t in range(20, 60):
            obs, r, d, _ = env.step(acts[t])
            for x, y in zip((obs, r, d), ref[t - 20]):
                np.testing.assert_array_equal(x.cpu().numpy(), y, err_msg=f"t={t}")
        got = np_state(env)
        for k in KEYS:
            np.testing.assert_array_equal(got[k], end[k], err_msg=k)
    other = make_env(EnvConfig(time_limit=25), N - 32, W, gpu, seed=21)
    with pytest.raises(BallEnvError, match="header"):
        other.load_state(dev_blob)
    with pytest.raises(ValueError, match="truncated"):
        env.load_state(host_blob[: host_blob.numel() - 16])
    env.status()
    env.close()
    other.close()


@pytest.mark.gpu
def test_save_state_host_blob_through_torch_save(gpu, tmp_path):
    """A host blob goes straight to torch.save with no manual synchronize (save_state returns it
    complete), and a blob loaded back from disk -- pageable memory, dropped right after
    load_state -- restores the state bit for bit."""
    from gym_ballenv_amd.config import EnvConfig
    N, W = 2048, 10
    env = make_env(EnvConfig(), N, W, gpu, seed=33)
    env.reset()
    acts = env.sample_actions(30, seed=9)
    for t in range(15):
        env.step(acts[t])
    want = np_state(env)
    path = tmp_path / "state.pt"
    torch.save(env.save_state("cpu"), path)
    for t in range(15, 30):
        env.step(acts[t])
    env.load_state(torch.load(path, weights_only=True))
    got = np_state(env)
    for k in KEYS:
        np.testing.assert_array_equal(got[k], want[k], err_msg=k)
    env.status()
    env.close()
