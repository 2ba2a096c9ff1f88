"""GPU: the autoreset pool (include/ballenv.h).

In Philox mode a reset into episode x is a pure function of (seed, global env id, x)
(gym_ballenv/envs/ballenv_env.py:113-167 with the counter layout of oracle/ballenv_oracle.c:186-228),
so pool_fill_kernel draws every env's resets into episodes e+1 and e+2 ahead of time and the
fixed-shape step kernels (step2_kernel at W=10, stepw_kernel at W=5, and the one-lane kernel of the
large batches at either W, forced here at small N by BALLENV_STEP_LPE / BALLENV_STEP5_LPE = 1) copy
the entry when the env finishes, drawing the reset inline only when the entry is stale.  These tests hold:
  * the entries themselves against the oracle's reset of the same env into the same episode;
  * stepping with the pool against stepping without it (BALLENV_POOL=0), every output and the
    state, bit for bit, through refills, stale entries, masked resets and load_state;
  * that a hit really copies the entry (a poisoned entry shows up in the state) and that a stale
    one is drawn inline (the oracle's state);
  * many resets per wave (TimeLimit 1: every env of every wave resets every step), hits and
    fallbacks mixed inside one wave, post-reset scalars against the oracle -- the cross-lane store
    ordering of the reset sinks.
"""
import os

import numpy as np
import pytest
import torch

from oracle import oracle
from test_gpu_parity import KEYS, assert_state_equal, make_env, np_state

pytestmark = pytest.mark.gpu

KERNEL = {10: "step2_kernel<10, 13, 5, true>", 5: "stepw_kernel<5, 13, 5, 8, true>",
          (10, 1): "be_kernel<10, 0, 13, 5, true>", (5, 1): "be_kernel<5, 0, 13, 5, true>"}


def _one_lane(monkeypatch, W, one):
    """one=True: the one-lane fixed-shape kernel at this W (read at be_create); returns KERNEL's key"""
    if one:
        monkeypatch.setenv("BALLENV_STEP_LPE" if W == 10 else "BALLENV_STEP5_LPE", "1")
        return (W, 1)
    return W


def _no_pool_env(cfg_py, N, W, dev, **kw):
    old = os.environ.get("BALLENV_POOL")
    os.environ["BALLENV_POOL"] = "0"
    try:
        return make_env(cfg_py, N, W, dev, **kw)
    finally:
        if old is None:
            del os.environ["BALLENV_POOL"]
        else:
            os.environ["BALLENV_POOL"] = old


def _rows_from_obs(row, W):
    """The pool's packed distinct window rows from an obs row (quirk Q1: distinct row k is window
    row k + 1): W = 10 three 10-bit rows per word, W = 5 four 5-bit rows in word 0."""
    cells = row[4:].reshape(W, W)
    rows = [int(sum(int(cells[k + 1, c]) << c for c in range(W))) for k in range(W - 1)]
    if W == 10:
        return [rows[0] | rows[1] << 10 | rows[2] << 20, rows[3] | rows[4] << 10 | rows[5] << 20,
                rows[6] | rows[7] << 10 | rows[8] << 20]
    return [rows[0] | rows[1] << 5 | rows[2] << 10 | rows[3] << 15, 0, 0]


def _u32(a):
    """packed (x, y) int16 pairs as the engine's u32 words, flattened"""
    return np.ascontiguousarray(a).view(np.uint32).reshape(-1)


@pytest.mark.parametrize("W", [10, 5])
def test_pool_entries_equal_the_oracle_reset(gpu, W):
    """After reset() every env's entries for episodes e+1 and e+2 are written, tagged, and equal the
    oracle's reset of that env into that episode: agent, goal, both distances, every obstacle and
    the new episode's window rows."""
    from gym_ballenv_amd.config import EnvConfig
    N, seed = 4096, 21
    cfg_py = EnvConfig()
    env = make_env(cfg_py, N, W, gpu, seed=seed)
    assert env.kernel_name("step") == KERNEL[W] and env.pool_bytes() > 0
    env.reset()
    ep = env.episode.cpu().numpy().view(np.uint32)
    rng = np.random.default_rng(W)
    for i in rng.choice(N, 24, replace=False):
        for x in (int(ep[i]) + 1, int(ep[i]) + 2):
            words, f64 = env.pool_entry(int(i), x & 1)
            cfg = cfg_py.to_abi(1, W, env_offset=int(i), seed=seed)
            st, out = oracle.new_state(cfg), oracle.new_out(cfg)
            st["episode"][:] = x - 1
            oracle.reset(cfg, st, out)
            assert words[0] == x, (i, x)
            assert words[3] & (1 << 30) and not words[3] & (1 << 31)
            assert words[1] == _u32(st["agent"])[0] and words[2] == _u32(st["goal"])[0]
            assert f64 == [st["prev_dist"][0], st["total_dist"][0]]
            np.testing.assert_array_equal(np.array(words[6:6 + 13], np.uint32), _u32(st["static_obs"]))
            np.testing.assert_array_equal(np.array(words[19:24], np.uint32), _u32(st["dyn_obs"]))
            want = _rows_from_obs(out["obs"][0], W)
            assert [words[3] & 0x3FFFFFFF, words[4], words[5]] == want, (i, x)
    env.close()


def _pair(cfg_py, N, W, dev, seed, key=None, **kw):
    key = W if key is None else key
    a = make_env(cfg_py, N, W, dev, seed=seed, **kw)
    b = _no_pool_env(cfg_py, N, W, dev, seed=seed, **kw)
    assert a.pool_bytes() > 0 and b.pool_bytes() == 0
    assert a.kernel_name("step") == KERNEL[key] and b.kernel_name("step") == KERNEL[key].replace("true>", "false>")
    return a, b


def _same_step(a, b, act, t):
    ra, rb = a.step(act, copy=True), b.step(act, copy=True)
    for x, y, name in zip(ra[:3], rb[:3], ("obs", "reward", "done")):
        assert torch.equal(x, y), f"t={t} {name}"
    for k in ra[3]:
        d = ra[2]
        if k in ("final_return", "final_len", "terminal_obs"):
            assert torch.equal(ra[3][k][d], rb[3][k][d]), f"t={t} {k}"
        else:
            assert torch.equal(ra[3][k], rb[3][k]), f"t={t} {k}"
    for k in KEYS:
        assert torch.equal(getattr(a, k), getattr(b, k)), f"t={t} state[{k}]"
    return int(ra[2].sum())


@pytest.mark.parametrize("W,N,period,one", [(10, 65536, 16, False), (10, 32768, 4, False), (5, 4096, 16, False),
                                            (5, 4096, 1, False), (10, 20000, 16, True), (5, 8192, 4, True)])
def test_pool_steps_equal_inline_resets(gpu, W, N, period, one, monkeypatch):
    """The pool's env against an env without it, same ids and seed: 240 steps at TimeLimit 40 from
    random ep_len phases (thousands of resets, refills every `period` steps, entries going stale in
    between), every output, the terminal obs and the state bit for bit; the stats slots equal.
    one=True: the one-lane kernel (N = 20000: a partial last block)."""
    from gym_ballenv_amd.config import EnvConfig
    cfg_py = EnvConfig(time_limit=40)
    a, b = _pair(cfg_py, N, W, gpu, seed=7, key=_one_lane(monkeypatch, W, one), terminal_obs=True)
    a.pool_set_period(period)
    a.reset()
    b.reset()
    lens = torch.randint(0, 40, (N,), dtype=torch.int32, device=gpu)
    a.ep_len.copy_(lens)
    b.ep_len.copy_(lens)
    acts = a.sample_actions(240, seed=8)
    resets = sum(_same_step(a, b, acts[t], t) for t in range(240))
    assert resets > 6 * N, resets
    assert torch.equal(a.stats_buf, b.stats_buf)
    a.status()
    b.status()
    a.close()
    b.close()


@pytest.mark.parametrize("W,one", [(10, False), (5, False), (10, True), (5, True)])
def test_pool_hit_copies_the_entry_and_stale_draws_inline(gpu, W, one, monkeypatch):
    """A hit copies the entry: a poisoned entry (valid tag, a moved agent) is what the env resets to.
    A stale entry (tag of another episode) is not used: the env resets to the oracle's state."""
    from gym_ballenv_amd.config import EnvConfig
    N, seed, j = 256, 9, 77
    cfg_py = EnvConfig(time_limit=1000)
    key = _one_lane(monkeypatch, W, one)
    env = make_env(cfg_py, N, W, gpu, seed=seed)
    assert env.kernel_name("step") == KERNEL[key]
    env.pool_set_period(0)
    env.reset()
    e = int(env.episode[j].item())
    words, f64 = env.pool_entry(j, (e + 1) & 1)
    poisoned = list(words)
    poisoned[1] = (7 & 0xFFFF) | (3 << 16)                     # agent (7, 3)
    env.pool_entry(j, (e + 1) & 1, write=(poisoned, f64))
    env.ep_len[j] = 999                                        # truncates on the next step
    env.step(torch.full((N,), 5, dtype=torch.uint8, device=gpu))
    assert env.episode[j].item() == e + 1 and env.ep_len[j].item() == 0
    assert env.agent[j].tolist() == [7, 3], "the step kernel did not copy the pool entry"
    # stale: entry e+2 re-tagged to another episode -> the inline draw, as the oracle's reset
    words2, f2 = env.pool_entry(j, (e + 2) & 1)
    assert words2[0] == e + 2
    stale = list(words2)
    stale[0] = e + 4
    stale[1] = (9 & 0xFFFF) | (4 << 16)
    env.pool_entry(j, (e + 2) & 1, write=(stale, f2))
    env.ep_len[j] = 999
    env.step(torch.full((N,), 5, dtype=torch.uint8, device=gpu))
    cfg = cfg_py.to_abi(1, W, env_offset=j, seed=seed)
    st, out = oracle.new_state(cfg), oracle.new_out(cfg)
    st["episode"][:] = e + 1
    oracle.reset(cfg, st, out)
    assert env.episode[j].item() == e + 2
    assert env.agent[j].tolist() == st["agent"][0].tolist() != [9, 4]
    np.testing.assert_array_equal(env.static_obs[:, j].cpu().numpy(), st["static_obs"][:, 0])
    env.status()
    env.close()


@pytest.mark.parametrize("W,N,one", [(10, 4096, False), (5, 2048, False), (10, 3000, True), (5, 2048, True)])
def test_pool_many_resets_per_wave_vs_oracle(gpu, W, N, one, monkeypatch):
    """TimeLimit 1: every env of every wave resets on every step.  No refills between steps, so step
    0 hits every entry (e+1), step 1 every e+2 entry; before step 2 a random half of the envs gets a
    fresh fill (others stay stale) and before step 3 a random third of the e+3 entries is invalidated
    -- hits and inline resets inside the same waves.  Every output and the whole state (post-reset
    ep_return / ep_len / prev_dist / total_dist included) equal the oracle after every step."""
    from gym_ballenv_amd.config import EnvConfig
    seed = 31
    cfg_py = EnvConfig(time_limit=1)
    key = _one_lane(monkeypatch, W, one)
    env = make_env(cfg_py, N, W, gpu, seed=seed)
    assert env.kernel_name("step") == KERNEL[key]
    env.pool_set_period(0)
    cfg = cfg_py.to_abi(N, W, seed=seed)
    st, out = oracle.new_state(cfg), oracle.new_out(cfg)
    env.reset()
    oracle.reset(cfg, st, out)
    assert_state_equal(env, st, "reset")
    acts = env.sample_actions(6, seed=seed)
    rng = np.random.default_rng(W)
    for t in range(6):
        if t == 2:
            env.pool_fill()                     # every env's e+1 / e+2 (e = 2 + episode after reset)
            for i in rng.choice(N, N // 2, replace=False):   # ... then half of the e+1 entries stale again
                e = int(env.episode[int(i)].item())
                words, f64 = env.pool_entry(int(i), (e + 1) & 1)
                words[0] = e + 7
                env.pool_entry(int(i), (e + 1) & 1, write=(words, f64))
        if t == 3:
            for i in rng.choice(N, N // 3, replace=False):
                e = int(env.episode[int(i)].item())
                words, f64 = env.pool_entry(int(i), (e + 1) & 1)
                words[3] &= ~(1 << 30)          # unwritten
                env.pool_entry(int(i), (e + 1) & 1, write=(words, f64))
        obs, reward, done, info = env.step(acts[t])
        oracle.step(cfg, st, out, actions=acts[t].cpu().numpy())
        assert out["done"].all()
        np.testing.assert_array_equal(obs.cpu().numpy(), out["obs"], err_msg=f"t={t} obs")
        np.testing.assert_array_equal(reward.cpu().numpy(), out["reward"], err_msg=f"t={t} reward")
        np.testing.assert_array_equal(info["final_return"].cpu().numpy(), out["final_return"], err_msg=f"t={t}")
        assert_state_equal(env, st, f"t={t}")
    env.status()
    env.close()


@pytest.mark.parametrize("W,one", [(10, False), (5, False), (10, True)])
def test_pool_masked_reset_and_load_state(gpu, W, one, monkeypatch):
    """Masked reset() and load_state() with the pool: both fill it for the state they leave (the
    entries need no invalidation -- each is a pure function of the env's id and episode), and the
    env then steps exactly as one without a pool; a reloaded blob replays its steps bit for bit."""
    from gym_ballenv_amd.config import EnvConfig
    N = 4096
    cfg_py = EnvConfig(time_limit=25)
    a, b = _pair(cfg_py, N, W, gpu, seed=13, key=_one_lane(monkeypatch, W, one))
    a.reset()
    b.reset()
    acts = a.sample_actions(90, seed=14)
    for t in range(20):
        _same_step(a, b, acts[t], t)
    mask = torch.rand(N, device=gpu) < 0.5
    a.reset(mask)
    b.reset(mask)
    for k in KEYS:
        assert torch.equal(getattr(a, k), getattr(b, k)), k
    blob = a.save_state()
    outs = []
    for t in range(20, 60):
        _same_step(a, b, acts[t], t)
        outs.append((a.obs.clone(), a.reward.clone(), a.done.clone()))
    a.load_state(blob)               # 40 steps back: episodes go back, the entries ahead stay valid
    b.load_state(blob)
    for t in range(20, 60):
        _same_step(a, b, acts[t], t)
        o = outs[t - 20]
        assert torch.equal(a.obs, o[0]) and torch.equal(a.reward, o[1]) and torch.equal(a.done, o[2]), t
    a.status()
    b.status()
    a.close()
    b.close()


def test_step_copy_semantics(gpu):
    """step() returns the env's output buffers, overwritten by the next step: a caller keeping
    per-step outputs (ball_cnn_ac3.py:610 appends rewards) must clone them, or ask copy=True (fresh
    tensors each call, as BallEnv.step returns a fresh array, ballenv_env.py:289).  50 steps kept
    both ways equal rollout() of the same actions from the same state; the un-cloned list aliases."""
    from gym_ballenv_amd.config import EnvConfig
    N, T = 2048, 50
    cfg_py = EnvConfig(time_limit=30)
    env = make_env(cfg_py, N, 10, gpu, seed=3)
    ref = make_env(cfg_py, N, 10, gpu, seed=3)
    env.reset()
    ref.reset()
    acts = env.sample_actions(T, seed=5)
    kept_copy, kept_clone, kept_alias = [], [], []
    for t in range(T):
        if t % 2:
            obs, reward, done, info = env.step(acts[t], copy=True)
            kept_copy.append((t, obs, reward, done, info["truncated"]))
        else:
            obs, reward, done, info = env.step(acts[t])
            kept_clone.append((t, obs.clone(), reward.clone(), done.clone(), info["truncated"].clone()))
        kept_alias.append(reward)
    r_obs, r_reward, r_done, r_info = ref.rollout(acts)
    for t, obs, reward, done, trunc in kept_copy + kept_clone:
        assert torch.equal(obs, r_obs[t]) and torch.equal(reward, r_reward[t]), t
        assert torch.equal(done, r_done[t]) and torch.equal(trunc, r_info["truncated"][t]), t
    # the un-cloned rewards of the even steps are all the env's one reward buffer, which now holds
    # the last step's rewards: keeping them without a clone loses every earlier step
    assert all(r is env.reward for t, r in enumerate(kept_alias) if t % 2 == 0)
    assert torch.equal(kept_alias[0], r_reward[T - 1]) and not torch.equal(kept_alias[0], r_reward[0])
    env.close()
    ref.close()
