"""GPU (HIP, gfx950) parity on the full default episode: the production kernels against the
oracle through goal changes and the TimeLimit.

The bench workload (EnvConfig() defaults, caller actions) runs the fixed-shape step kernel
(step2_kernel<10, 13, 5> at W=10 up to 98 304 envs, be_kernel<10, 0, 13, 5> past that,
stepw_kernel<5, 13, 5, 8> at W=5 up to 64 x CUs envs), the fused be_rollout kernel
and the fused be_policy_rollout kernel.
Each has its own goal re-pick (newGoalList for pairwise-distinct goals, ballenv_env.py:339-353)
and its own `ep_len mod (goal_change+1)` counter arithmetic, and all of them fold the gym
TimeLimit(1000) (gym_ballenv/__init__.py:7) plus the autoreset into the step.  From a fresh
reset the first goal change is 51 steps away and the TimeLimit 1000.  These tests therefore
start every env at a random ep_len -- all goal-change phases, with a quarter of the envs at
990..999 so that TimeLimit truncations happen within a few steps -- and compare
every per-step output and the state with the C oracle (pinned to the reference's golden
vectors in test_oracle_golden.py) on a 2048-env slice keyed by global env id.
"""
import numpy as np
import pytest
import torch

from oracle import oracle
from test_gpu_parity import KEYS, make_env, np_state

pytestmark = pytest.mark.gpu

SLICE = 2048


def fixed_step_kernel(W, N=0):
    """The step kernel pick_kernel selects at the defaults with caller actions: step2_kernel at
    W=10 up to 96 x 4 x CUs envs, stepw_kernel (8 lanes per env) at W=5 up to 64 x CUs envs, the
    one-lane fixed-shape kernel otherwise."""
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    if W == 10 and N <= 96 * 4 * cus:
        return "step2_kernel<10, 13, 5, true>"
    if W == 5 and N <= 64 * cus:
        return "stepw_kernel<5, 13, 5, 8, true>"
    # the one-lane kernel takes the autoreset pool up to two waves per SIMD (128 x 4 x CUs envs)
    return f"be_kernel<{W}, 0, 13, 5, {'true' if N <= 2 * 64 * 4 * cus else 'false'}>"


def _random_lens(N, rng, limit=1000):
    lens = rng.integers(0, limit, N).astype(np.int32)
    near = rng.random(N) < 0.25
    lens[near] = rng.integers(max(0, limit - 10), limit, int(near.sum()))
    return lens


def _slice_state(st, a, k):
    out = {}
    for key, v in st.items():
        out[key] = v[:, a:a + k] if key in ("static_obs", "dyn_obs", "dyn_goal") else v[a:a + k]
    return out


def _setup(cfg_py, N, W, dev, a, k, seed, rng, terminal=True):
    """GPU env (N envs) and an oracle on global envs [a, a+k), both reset and then moved to the
    same random ep_len phase."""
    env = make_env(cfg_py, N, W, dev, seed=seed, terminal_obs=terminal)
    cfg = cfg_py.to_abi(k, W, env_offset=a, seed=seed)
    st = oracle.new_state(cfg)
    out = oracle.new_out(cfg, terminal=terminal)
    oracle.reset(cfg, st, out)
    env.reset()
    lens = _random_lens(N, rng, cfg_py.time_limit or 1000)
    env.ep_len.copy_(torch.from_numpy(lens).to(dev))
    st["ep_len"][:] = lens[a:a + k]
    got = _slice_state(np_state(env), a, k)
    for key in KEYS:
        np.testing.assert_array_equal(got[key], st[key], err_msg=f"after reset: {key}")
    return env, cfg, st, out


def _check_step(t, a, k, out, obs, reward, done, trunc, fret, flen, term=None):
    sl = slice(a, a + k)
    d = done[sl].cpu().numpy()
    np.testing.assert_array_equal(reward[sl].cpu().numpy(), out["reward"], err_msg=f"reward t={t}")
    np.testing.assert_array_equal(d, out["done"].astype(bool), err_msg=f"done t={t}")
    np.testing.assert_array_equal(trunc[sl].cpu().numpy(), out["truncated"].astype(bool), err_msg=f"truncated t={t}")
    np.testing.assert_array_equal(obs[sl].cpu().numpy(), out["obs"], err_msg=f"obs t={t}")
    np.testing.assert_array_equal(fret[sl].cpu().numpy()[d], out["final_return"][d], err_msg=f"final_return t={t}")
    np.testing.assert_array_equal(flen[sl].cpu().numpy()[d], out["final_len"][d], err_msg=f"final_len t={t}")
    if term is not None:
        np.testing.assert_array_equal(term[sl].cpu().numpy()[d], out["terminal_obs"][d], err_msg=f"terminal_obs t={t}")
    return int(out["truncated"].sum())


def _check_state(env, st, a, k, msg):
    got = _slice_state(np_state(env), a, k)
    for key in KEYS:
        np.testing.assert_array_equal(got[key], st[key], err_msg=f"{msg}: state[{key}]")


@pytest.mark.parametrize("W,N,a", [(10, 65536, 40960), (5, 4096, 1024), (10, 3000, 952), (10, 262144, 200000),
                                   (10, 32768, 20000)])
def test_step_kernel_default_episode(gpu, W, N, a):
    """be_step (fixed-shape kernel) at the defaults -- goal change every 51 steps, TimeLimit
    1000, autoreset -- bit-exact against the oracle over 120 steps (>= 2 goal changes per env
    that survives), including truncations from the TimeLimit."""
    from gym_ballenv_amd.config import EnvConfig
    cfg_py = EnvConfig()
    assert cfg_py.time_limit == 1000 and cfg_py.goal_change_step == 50
    rng = np.random.default_rng(W * 7 + N)
    k = min(SLICE, N - a)
    env, cfg, st, out = _setup(cfg_py, N, W, gpu, a, k, seed=0xBA11, rng=rng)
    assert env.kernel_name("step") == fixed_step_kernel(W, N)
    acts = env.sample_actions(120, seed=0xBA11)
    n_trunc = n_change = 0
    for t in range(120):
        out["terminal_obs"][:] = 0
        env.terminal_obs.zero_()
        g0 = st["dyn_goal"].copy()
        oracle.step(cfg, st, out, actions=acts[t, a:a + k].cpu().numpy())
        n_change += int((st["dyn_goal"] != g0).any(0).sum())
        obs, reward, done, info = env.step(acts[t])
        n_trunc += _check_step(t, a, k, out, obs, reward, done, info["truncated"], info["final_return"],
                               info["final_len"], info["terminal_obs"])
        _check_state(env, st, a, k, f"t={t}")
    assert n_trunc > 0 and n_change > 0, (n_trunc, n_change)
    env.status()
    env.close()


@pytest.mark.parametrize("W", [10, 5])
def test_step_kernel_top_of_id_space(gpu, W):
    """A maximum-size case: 2^22 envs whose global ids end at the top of the 32-bit id space
    (env_offset = 2^32 - 2^22, be_config_check's limit), the one-lane fixed-shape kernel; the
    last 2048 envs (ids 2^32 - 2048 .. 2^32 - 1) bit-exact against the oracle over 40
    default-config steps from random ep_len phases, truncations and goal changes included --
    the Philox keys' 32-bit id arithmetic and index arithmetic past 2^24 envs."""
    from gym_ballenv_amd.config import EnvConfig
    from test_gpu_parity import KEYS as SK
    cfg_py = EnvConfig()
    N = 1 << 22
    off, k = (1 << 32) - N, SLICE
    a = N - k
    env = make_env(cfg_py, N, W, gpu, seed=0xBA11, env_offset=off, terminal_obs=True)
    assert env.kernel_name("step") == fixed_step_kernel(W, N) == f"be_kernel<{W}, 0, 13, 5, false>"
    cfg = cfg_py.to_abi(k, W, env_offset=off + a, seed=0xBA11)
    st = oracle.new_state(cfg)
    out = oracle.new_out(cfg, terminal=True)
    oracle.reset(cfg, st, out)
    env.reset()
    lens = _random_lens(N, np.random.default_rng(W))
    env.ep_len.copy_(torch.from_numpy(lens).to(gpu))
    st["ep_len"][:] = lens[a:]

    def check_slice(msg):   # the slice only: the whole 2^22-env state is ~0.5 GB
        for key in SK:
            v = getattr(env, key)
            got = (v[:, a:] if key in ("static_obs", "dyn_obs", "dyn_goal") else v[a:]).cpu().numpy()
            want = st[key].view(np.int32) if key == "episode" else st[key]
            np.testing.assert_array_equal(got, want, err_msg=f"{msg}: state[{key}]")

    check_slice("after reset")
    acts = env.sample_actions(40, seed=0xBA11)
    n_trunc = 0
    for t in range(40):
        out["terminal_obs"][:] = 0
        env.terminal_obs.zero_()
        oracle.step(cfg, st, out, actions=acts[t, a:].cpu().numpy())
        obs, reward, done, info = env.step(acts[t])
        n_trunc += _check_step(t, a, k, out, obs, reward, done, info["truncated"], info["final_return"],
                               info["final_len"], info["terminal_obs"])
        check_slice(f"t={t}")
    assert n_trunc > 0
    env.status()
    env.close()


def test_rollout_kernel_top_of_id_space(gpu):
    """be_rollout (the fused random-action rollout, one-lane rollout_kernel) at the top of the 32-bit
    global-id space: 2^21 envs ending at id 2^32 - 1, two launches of 20 steps; the last 2048 envs'
    per-step outputs and state bit-exact against the oracle, truncations and goal changes included."""
    from gym_ballenv_amd.config import EnvConfig
    from test_gpu_parity import KEYS as SK
    cfg_py = EnvConfig()
    N, W = 1 << 21, 10
    off, k = (1 << 32) - N, SLICE
    a = N - k
    env = make_env(cfg_py, N, W, gpu, seed=0x5EED, env_offset=off, terminal_obs=True)
    assert env.kernel_name("rollout") == "rollout_kernel<10, 13, 5, 0, 1, 10>"
    cfg = cfg_py.to_abi(k, W, env_offset=off + a, seed=0x5EED)
    st = oracle.new_state(cfg)
    out = oracle.new_out(cfg, terminal=True)
    oracle.reset(cfg, st, out)
    env.reset()
    lens = _random_lens(N, np.random.default_rng(21))
    env.ep_len.copy_(torch.from_numpy(lens).to(gpu))
    st["ep_len"][:] = lens[a:]
    acts = env.sample_actions(40, seed=23)
    n_trunc, t0 = 0, 0
    for K in (20, 20):
        obs, reward, done, info = env.rollout(acts[t0:t0 + K])
        for j in range(K):
            t = t0 + j
            out["terminal_obs"][:] = 0
            oracle.step(cfg, st, out, actions=acts[t, a:].cpu().numpy())
            n_trunc += _check_step(t, a, k, out, obs[j], reward[j], done[j], info["truncated"][j],
                                   info["final_return"][j], info["final_len"][j], info["terminal_obs"][j])
        t0 += K
        for key in SK:
            v = getattr(env, key)
            got = (v[:, a:] if key in ("static_obs", "dyn_obs", "dyn_goal") else v[a:]).cpu().numpy()
            want = st[key].view(np.int32) if key == "episode" else st[key]
            np.testing.assert_array_equal(got, want, err_msg=f"after step {t0}: state[{key}]")
    assert n_trunc > 0
    env.status()
    env.close()


def test_step_kernel_time_limit_boundary(gpu):
    """Every env starts at ep_len 995..999: the TimeLimit truncates the survivors within five
    steps and the autoreset starts their next episode (ep_len 999 -> done, ep_len 0)."""
    from gym_ballenv_amd.config import EnvConfig
    cfg_py = EnvConfig()
    N, W = 4096, 10
    rng = np.random.default_rng(3)
    env, cfg, st, out = _setup(cfg_py, N, W, gpu, 0, N, seed=99, rng=rng)
    lens = rng.integers(995, 1000, N).astype(np.int32)
    env.ep_len.copy_(torch.from_numpy(lens).to(gpu))
    st["ep_len"][:] = lens
    acts = torch.full((N,), 5, dtype=torch.uint8, device=gpu)    # (0, 0): stay put, fewer collisions
    n_trunc = 0
    for t in range(8):
        out["terminal_obs"][:] = 0
        env.terminal_obs.zero_()
        oracle.step(cfg, st, out, actions=acts.cpu().numpy())
        obs, reward, done, info = env.step(acts)
        n_trunc += _check_step(t, 0, N, out, obs, reward, done, info["truncated"], info["final_return"],
                               info["final_len"], info["terminal_obs"])
        _check_state(env, st, 0, N, f"t={t}")
    assert n_trunc > N // 4, n_trunc
    assert (env.ep_len.cpu().numpy() < 10).all()
    env.status()
    env.close()


@pytest.mark.parametrize("G", [0, 1, 3, 5, 7, 11, 50])
@pytest.mark.parametrize("W", [10, 5])
def test_goal_change_steps_vs_oracle(gpu, G, W):
    """Short goal-change periods with caller actions (so the fixed-shape kernel runs): every
    env goes through many goal re-picks (pick + (pick >= current goal)) against the oracle."""
    from gym_ballenv_amd.config import EnvConfig
    cfg_py = EnvConfig(goal_change_step=G)
    N = 4096
    rng = np.random.default_rng(100 + G)
    env, cfg, st, out = _setup(cfg_py, N, W, gpu, 0, N, seed=G + 1, rng=rng)
    assert env.kernel_name("step") == fixed_step_kernel(W)
    acts = env.sample_actions(30, seed=G)
    n_change = 0
    for t in range(30):
        out["terminal_obs"][:] = 0
        env.terminal_obs.zero_()
        g0 = st["dyn_goal"].copy()
        oracle.step(cfg, st, out, actions=acts[t].cpu().numpy())
        n_change += int((st["dyn_goal"] != g0).sum())
        obs, reward, done, info = env.step(acts[t])
        _check_step(t, 0, N, out, obs, reward, done, info["truncated"], info["final_return"], info["final_len"],
                    info["terminal_obs"])
        _check_state(env, st, 0, N, f"G={G} t={t}")
    assert n_change > 0
    env.status()
    env.close()


@pytest.mark.parametrize("W,N,a,G", [(10, 65536, 8192, 50), (5, 4096, 2048, 50), (10, 4096, 0, 3)])
def test_rollout_kernel_default_episode(gpu, W, N, a, G):
    """be_rollout (the fused random-action rollout) against the oracle through goal changes and
    TimeLimit truncations: 120 steps as chunks of 50 + 70."""
    from gym_ballenv_amd.config import EnvConfig
    cfg_py = EnvConfig(goal_change_step=G)
    rng = np.random.default_rng(W + N + G)
    k = min(SLICE, N - a)
    env, cfg, st, out = _setup(cfg_py, N, W, gpu, a, k, seed=0x5EED, rng=rng)
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    want = "rolloutw_kernel<5, 13, 5, 8>" if W == 5 and N <= 64 * cus else f"rollout_kernel<{W}, 13, 5, 0, 1, 10>"
    assert env.kernel_name("rollout") == want
    acts = env.sample_actions(120, seed=17)
    n_trunc, t0 = 0, 0
    for K in (50, 70):
        obs, reward, done, info = env.rollout(acts[t0:t0 + K])
        for j in range(K):
            t = t0 + j
            out["terminal_obs"][:] = 0
            oracle.step(cfg, st, out, actions=acts[t, a:a + k].cpu().numpy())
            n_trunc += _check_step(t, a, k, out, obs[j], reward[j], done[j], info["truncated"][j],
                                   info["final_return"][j], info["final_len"][j], info["terminal_obs"][j])
        t0 += K
        _check_state(env, st, a, k, f"after step {t0}")
    assert G != 50 or n_trunc > 0
    env.status()
    env.close()


@pytest.mark.parametrize("W,N,a", [(10, 65536, 16384), (5, 4096, 0)])
def test_policy_rollout_default_episode(gpu, W, N, a):
    """be_policy_rollout (select_action + step fused) against the oracle stepped with the
    actions the kernel drew: rewards, dones, recorded obs and the state after 2 x 60 steps,
    through goal changes and TimeLimit truncations.  (The action draw itself is checked
    against PyTorch in test_gpu_policy.py / test_gpu_rollout.py.)"""
    from gym_ballenv_amd.config import EnvConfig
    from gym_ballenv_amd.policy import Policy, reference_weights
    from gym_ballenv_amd.rollout import Rollout
    cfg_py = EnvConfig()
    rng = np.random.default_rng(W * 13)
    k = min(SLICE, N - a)
    env, cfg, st, out = _setup(cfg_py, N, W, gpu, a, k, seed=0xACE, rng=rng, terminal=False)
    path = reference_weights(W)
    torch.manual_seed(0)
    pol = Policy.from_npz(path, W) if path else Policy(W)
    T = 60
    ro = Rollout(env, pol, horizon=T, backend="fused", record_obs=True, seed=0x5E1EC7, chunk=T)
    n_trunc = 0
    for h in range(2):
        ro.run_eager()
        acts = ro.actions[:, a:a + k].cpu().numpy()
        np.testing.assert_array_equal(ro.obs[0, a:a + k].cpu().numpy(), out["obs"] if h else ro.obs[0, a:a + k].cpu().numpy())
        for t in range(T):
            oracle.step(cfg, st, out, actions=acts[t])
            np.testing.assert_array_equal(ro.rewards[t, a:a + k].cpu().numpy(), out["reward"], err_msg=f"h={h} t={t}")
            np.testing.assert_array_equal(ro.dones[t, a:a + k].cpu().numpy(), out["done"].astype(bool))
            np.testing.assert_array_equal(ro.obs[t + 1, a:a + k].cpu().numpy(), out["obs"], err_msg=f"obs h={h} t={t}")
            n_trunc += int(out["truncated"].sum())
        _check_state(env, st, a, k, f"horizon {h}")
        np.testing.assert_array_equal(env.obs[a:a + k].cpu().numpy(), out["obs"])
    assert n_trunc > 0
    env.status()
    ro.close()
    env.close()


def test_step_kernel_dispatch_by_batch(gpu, monkeypatch):
    """W=10 steps on step2_kernel up to 1.5 waves per SIMD of one-lane work (96 x 4 x CUs envs,
    98 304 on a 256-CU MI355X) and on the one-lane kernel past it; BALLENV_STEP_LPE overrides."""
    from gym_ballenv_amd.config import EnvConfig
    monkeypatch.delenv("BALLENV_STEP_LPE", raising=False)
    cus = torch.cuda.get_device_properties(gpu).multi_processor_count
    cut = 96 * 4 * cus
    for N, name in ((cut, "step2_kernel<10, 13, 5, true>"), (cut + 64, "be_kernel<10, 0, 13, 5, true>")):
        e = make_env(EnvConfig(), N, 10, gpu, seed=1)
        assert e.kernel_name("step") == name, (N, cus)
        e.close()
    monkeypatch.setenv("BALLENV_STEP_LPE", "2")
    e = make_env(EnvConfig(), cut + 64, 10, gpu, seed=1)
    assert e.kernel_name("step") == "step2_kernel<10, 13, 5, true>"
    e.close()


@pytest.mark.parametrize("N,tl,f32", [(20000, 20, False), (65536, 1000, False), (1000, 7, False), (4000, 20, True),
                                     (32768, 1000, False), (1, 7, False), (33, 7, True)])
def test_step2_equals_one_lane_kernel(gpu, N, tl, f32, monkeypatch):
    """step2_kernel (two lanes per env) equals the one-lane fixed-shape kernel bit for bit --
    obs, reward, done, truncated, final return / length, terminal obs, the state and the
    stats slots -- through mass truncation (tl=20: every env of every wave resets on the same
    steps) and at the defaults from random episode phases (N=32768: config 4's per-GPU shard at
    8 GPUs); N=20000 / 1000 leave partial blocks, N=1 / 33 a lone env and a one-env last wave."""
    from gym_ballenv_amd.config import EnvConfig
    cfg_py = EnvConfig(time_limit=tl)
    W = 10
    envs = []
    for lpe in ("2", "1"):
        monkeypatch.setenv("BALLENV_STEP_LPE", lpe)
        envs.append(make_env(cfg_py, N, W, gpu, seed=31, terminal_obs=True, obs_f32=f32))
    monkeypatch.delenv("BALLENV_STEP_LPE")
    assert envs[0].kernel_name("step") == "step2_kernel<10, 13, 5, true>"
    assert envs[1].kernel_name("step") == "be_kernel<10, 0, 13, 5, true>"
    lens = torch.from_numpy(_random_lens(N, np.random.default_rng(N), tl)).to(gpu)
    for e in envs:
        e.reset()
        e.ep_len.copy_(lens)
    acts = envs[0].sample_actions(45, seed=9)
    n_done = 0
    for t in range(45):
        for e in envs:
            e.terminal_obs.zero_()
        res = [e.step(acts[t]) for e in envs]
        d = res[0][2].cpu().numpy()
        n_done += int(d.sum())
        s0 = np_state(envs[0])
        for v in (1,):
            for a, b in zip(res[0][:3], res[v][:3]):
                np.testing.assert_array_equal(a.cpu().numpy(), b.cpu().numpy(), err_msg=f"variant {v} t={t}")
            for key in ("truncated", "terminal_obs"):
                np.testing.assert_array_equal(res[0][3][key].cpu().numpy(), res[v][3][key].cpu().numpy(), err_msg=key)
            if f32:   # step2_kernel's f32 copy-out (copy_out<64>) against the one-lane kernel's and the u8 obs
                np.testing.assert_array_equal(envs[0].obs_f32.cpu().numpy(), envs[v].obs_f32.cpu().numpy())
                np.testing.assert_array_equal(envs[0].obs_f32.cpu().numpy(), res[0][0].cpu().numpy().astype(np.float32))
            for key in ("final_return", "final_len"):
                np.testing.assert_array_equal(res[0][3][key].cpu().numpy()[d], res[v][3][key].cpu().numpy()[d])
            s1 = np_state(envs[v])
            for k in KEYS:
                np.testing.assert_array_equal(s0[k], s1[k], err_msg=f"variant {v} t={t} {k}")
    for v in (1,):
        np.testing.assert_array_equal(envs[0].stats_buf.cpu().numpy(), envs[v].stats_buf.cpu().numpy())
    assert n_done > 0
    for e in envs:
        e.status()
        e.close()


@pytest.mark.parametrize("r_obs", [22, 23])
def test_step2_span_table_radius_bound(gpu, r_obs):
    """step2_kernel rasterises from a 64-bit row-span table, which holds W-1+2R <= 63 (R <= 27 at
    W=10; the default R is 25).  R = 27 (the widest table) is bit-exact against the oracle; at R = 28
    the dispatch takes the one-lane fixed-shape kernel, also bit-exact."""
    from gym_ballenv_amd.config import EnvConfig
    cfg_py = EnvConfig(radius_obstacle=r_obs, time_limit=40)
    N, a, k, W = 8192, 4096, SLICE, 10
    rng = np.random.default_rng(r_obs)
    env, cfg, st, out = _setup(cfg_py, N, W, gpu, a, k, seed=0x5A, rng=rng)
    assert env.kernel_name("step") == ("step2_kernel<10, 13, 5, true>" if r_obs + 5 <= 27 else "be_kernel<10, 0, 13, 5, true>")
    acts = env.sample_actions(60, seed=0x5A)
    lit = 0
    for t in range(60):
        out["terminal_obs"][:] = 0
        env.terminal_obs.zero_()
        oracle.step(cfg, st, out, actions=acts[t, a:a + k].cpu().numpy())
        obs, reward, done, info = env.step(acts[t])
        _check_step(t, a, k, out, obs, reward, done, info["truncated"], info["final_return"], info["final_len"],
                    info["terminal_obs"])
        _check_state(env, st, a, k, f"t={t}")
        lit += int((out["obs"][:, 4:] != 0).any(1).sum())
    assert lit > 0
    env.status()
    env.close()


def test_step_n_equals_step_calls(gpu):
    """be_step_n (K launches queued by one call) leaves the same state, last-step outputs and
    stats slots as K be_step calls."""
    from gym_ballenv_amd.config import EnvConfig
    N, W, K = 6000, 10, 37
    envs = [make_env(EnvConfig(), N, W, gpu, seed=5) for _ in range(2)]
    lens = torch.from_numpy(_random_lens(N, np.random.default_rng(1))).to(gpu)
    for e in envs:
        e.reset()
        e.ep_len.copy_(lens)
    acts = envs[0].sample_actions(K, seed=2)
    for t in range(K):
        ra = envs[0].step(acts[t])
    rb = envs[1].step_n(acts)
    for x, y in zip(ra[:3], rb[:3]):
        np.testing.assert_array_equal(x.cpu().numpy(), y.cpu().numpy())
    sa, sb = np_state(envs[0]), np_state(envs[1])
    for k in KEYS:
        np.testing.assert_array_equal(sa[k], sb[k], err_msg=k)
    np.testing.assert_array_equal(envs[0].stats_buf.cpu().numpy(), envs[1].stats_buf.cpu().numpy())
    for e in envs:
        e.status()
        e.close()


@pytest.mark.parametrize("N,tl,f32", [(4096, 1000, False), (4096, 20, False), (1000, 7, True), (20000, 20, False),
                                     (1, 7, False), (33, 7, True)])
def test_stepw_equals_one_lane_kernel(gpu, N, tl, f32, monkeypatch):
    """stepw_kernel (W=5, 8 and 4 lanes per env, 32-env blocks with a last-wave stats fold) equals
    the one-lane fixed-shape kernel bit for bit -- obs (u8 and f32), reward, done, truncated,
    final return / length, terminal obs, the state and the stats slots -- through mass truncation
    (tl=20 / 7: every env of every wave resets on the same steps) and at the defaults from random
    episode phases; N=1000 / 20000 leave partial blocks and a partial last wave, N=1 / 33 a lone env and a
    one-env last block."""
    from gym_ballenv_amd.config import EnvConfig
    cfg_py = EnvConfig(time_limit=tl)
    W = 5
    envs = []
    for lpe in ("1", "8", "4"):
        monkeypatch.setenv("BALLENV_STEP5_LPE", lpe)
        envs.append(make_env(cfg_py, N, W, gpu, seed=77, terminal_obs=True, obs_f32=f32))
    monkeypatch.delenv("BALLENV_STEP5_LPE")
    assert [e.kernel_name("step") for e in envs] == ["be_kernel<5, 0, 13, 5, true>", "stepw_kernel<5, 13, 5, 8, true>",
                                                     "stepw_kernel<5, 13, 5, 4, true>"]
    lens = torch.from_numpy(_random_lens(N, np.random.default_rng(N + tl), tl)).to(gpu)
    for e in envs:
        e.reset()
        e.ep_len.copy_(lens)
    acts = envs[0].sample_actions(45, seed=19)
    n_done = 0
    for t in range(45):
        for e in envs:
            e.terminal_obs.zero_()
        res = [e.step(acts[t]) for e in envs]
        d = res[0][2].cpu().numpy()
        n_done += int(d.sum())
        s0 = np_state(envs[0])
        for v in (1, 2):
            for a, b in zip(res[0][:3], res[v][:3]):
                np.testing.assert_array_equal(a.cpu().numpy(), b.cpu().numpy(), err_msg=f"variant {v} t={t}")
            for key in ("truncated", "terminal_obs"):
                np.testing.assert_array_equal(res[0][3][key].cpu().numpy(), res[v][3][key].cpu().numpy(), err_msg=key)
            for key in ("final_return", "final_len"):
                np.testing.assert_array_equal(res[0][3][key].cpu().numpy()[d], res[v][3][key].cpu().numpy()[d])
            if f32:
                np.testing.assert_array_equal(envs[0].obs_f32.cpu().numpy(), envs[v].obs_f32.cpu().numpy())
            s1 = np_state(envs[v])
            for k in KEYS:
                np.testing.assert_array_equal(s0[k], s1[k], err_msg=f"variant {v} t={t} {k}")
    for v in (1, 2):
        np.testing.assert_array_equal(envs[0].stats_buf.cpu().numpy(), envs[v].stats_buf.cpu().numpy())
    assert n_done > 0
    for e in envs:
        e.status()
        e.close()


@pytest.mark.parametrize("W,N", [(10, 4096), (5, 4096), (10, 131072)])
def test_q9_resample_config_vs_oracle(gpu, W, N):
    """A config where a reset CAN re-sample the agent (agent strip y < 490 overlaps the goal strip,
    ballenv_env.py:121-126, quirk Q9: state[2] keeps the pre-resample distance): the fixed-shape
    kernels match the oracle through many such resets (time limit 12) on a 2048-env slice."""
    from gym_ballenv_amd.config import EnvConfig
    cfg_py = EnvConfig(strip_agent_y=490, time_limit=12)
    rng = np.random.default_rng(W + N)
    a = N - SLICE
    env, cfg, st, out = _setup(cfg_py, N, W, gpu, a, SLICE, seed=0x99, rng=rng)
    assert env.kernel_name("step") == fixed_step_kernel(W, N)
    acts = env.sample_actions(40, seed=3)
    q9 = 0
    for t in range(40):
        out["terminal_obs"][:] = 0
        env.terminal_obs.zero_()
        oracle.step(cfg, st, out, actions=acts[t, a:].cpu().numpy())
        q9 += int((st["ep_len"] == 0).sum() and (st["prev_dist"] != st["total_dist"]).sum())
        obs, reward, done, info = env.step(acts[t])
        _check_step(t, a, SLICE, out, obs, reward, done, info["truncated"], info["final_return"], info["final_len"],
                    info["terminal_obs"])
        _check_state(env, st, a, SLICE, f"t={t}")
    assert q9 > 0, "no reset re-sampled the agent"
    env.status()
    env.close()


def test_prev_dist_recompute_equals_read(gpu, monkeypatch):
    """At the defaults no reset can re-sample the agent, so prev_dist == calc_dist(goal, agent) and
    the fixed-shape kernels may recompute it instead of reading it (BALLENV_PREV_READ=0, an A/B
    option: slower): the same trajectory bit for bit (65 536 envs, W=10 / 4 096, W=5)."""
    from gym_ballenv_amd.config import EnvConfig
    for N, W in ((65536, 10), (4096, 5)):
        envs = []
        for v in ("0", None):
            if v:
                monkeypatch.setenv("BALLENV_PREV_READ", v)
            else:
                monkeypatch.delenv("BALLENV_PREV_READ", raising=False)
            envs.append(make_env(EnvConfig(), N, W, gpu, seed=41))
        lens = torch.from_numpy(_random_lens(N, np.random.default_rng(5))).to(gpu)
        for e in envs:
            e.reset()
            e.ep_len.copy_(lens)
        acts = envs[0].sample_actions(60, seed=8)
        for t in range(60):
            r0, r1 = (e.step(acts[t]) for e in envs)
            for x, y in zip(r0[:3], r1[:3]):
                np.testing.assert_array_equal(x.cpu().numpy(), y.cpu().numpy(), err_msg=f"N={N} t={t}")
        s0, s1 = np_state(envs[0]), np_state(envs[1])
        for k in KEYS:
            np.testing.assert_array_equal(s0[k], s1[k], err_msg=k)
        for e in envs:
            e.status()
            e.close()


def test_fixed_kernels_batch_size_bound(gpu):
    """The fixed-shape kernels address per-env arrays as a uniform base + a 32-bit byte offset, so the
    dispatcher takes them only below 2^29 envs (FIX_MAX_ENVS: element i of an 8-byte array); at 2^29
    the generic kernels (64-bit indexing) run.  Contexts only -- no state is allocated here."""
    import ctypes as C
    from gym_ballenv_amd import _abi
    from gym_ballenv_amd.config import EnvConfig
    lib = _abi.lib()
    dev = torch.device(gpu).index or 0
    names = {}
    for n in ((1 << 29) - 1, 1 << 29):
        cfg = EnvConfig().to_abi(n, 10)
        ctx = C.c_void_p()
        _abi.check(lib.be_create(C.byref(cfg), dev, C.byref(ctx)))
        try:
            names[n] = (lib.be_kernel_name(ctx, 0).decode(), lib.be_kernel_name(ctx, 2))   # rollout: NULL = loop
        finally:
            lib.be_destroy(ctx)
    assert names[(1 << 29) - 1][0] == "be_kernel<10, 0, 13, 5, false>", names   # (past 2^22 envs: no pool)
    assert names[1 << 29][0] == "be_kernel<10, 0, 0, 0, false>", names
    assert names[1 << 29][1] is None or b"13, 5" not in names[1 << 29][1], names
