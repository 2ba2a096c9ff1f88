"""The createBoard physics profile: ballenv_pygame.createBoard
reset/step/calc_reward + featureExtractor, against golden vectors made by running the
reference (tests/golden/make_golden_board.py) -- the C oracle on the CPU, and
BatchedBoard (csrc/board.hip) on the GPU.

Bar: positions, distances, rewards, returns and done bit-exact (f64, same operation
order); features exact except the social-force sum f[18] (exp / hypot / acos are 1-ulp
library functions on every side, so its f64 sums differ by ~1e-16 relative): at most 1 ulp
of f32 apart.
"""
import numpy as np
import pytest
import torch

from helpers import load
from oracle import oracle


def cfg_for(n, ns):
    import ctypes as C
    from gym_ballenv_amd import _abi
    c = _abi.BeBoardConfig()
    _abi.lib().be_board_config_default(C.byref(c), n, ns)
    return c


def f32_ulps(a, b):
    """|a - b| in units in the last place of f32 (ordered integer distance; +0 == -0)."""
    def key(x):
        i = np.ascontiguousarray(x, np.float32).view(np.int32).astype(np.int64)
        return np.where(i < 0, -(i & 0x7FFFFFFF), i)
    return np.abs(key(a) - key(b))


def check_features(got, want, msg=""):
    got, want = np.asarray(got, np.float32), np.asarray(want, np.float32)
    mask = np.ones(20, bool)
    mask[18] = False
    np.testing.assert_array_equal(got[..., mask], want[..., mask], err_msg=msg)
    assert np.isfinite(got[..., 18]).all() and np.isfinite(want[..., 18]).all(), msg
    u = f32_ulps(got[..., 18], want[..., 18])
    assert u.max() <= 1, f"{msg}: f[18] {int(u.max())} f32 ulps apart ({int((u > 0).sum())} of {u.size} differ)"


def fixture(prefix):
    fx = load("board")
    return {k[len(prefix) + 1:]: v for k, v in fx.items() if k.startswith(prefix + "_")}


@pytest.mark.parametrize("prefix", ["a", "b"])
def test_oracle_board_golden(prefix):
    g = fixture(prefix)
    E, T = g["actions"].shape
    ns = g["init_static"].shape[1]
    cfg = cfg_for(E, ns)
    st = oracle.board_new_state(cfg)
    tape = g["reset_tape"].T[: int(g["reset_used"].max())]
    status, f = oracle.board_reset(cfg, st, np.nan_to_num(tape))
    assert status == 0
    np.testing.assert_array_equal(st["agent"], g["init_agent"])
    np.testing.assert_array_equal(st["goal"], g["init_goal"])
    np.testing.assert_array_equal(st["dist"], g["init_dist"])
    np.testing.assert_array_equal(st["total_dist"], g["init_total"])
    np.testing.assert_array_equal(st["static_obs"].transpose(1, 0, 2), g["init_static"])
    check_features(f, g["init_feat"], "reset")
    for t in range(T):
        r, d, f = oracle.board_step(cfg, st, actions=g["actions"][:, t])
        np.testing.assert_array_equal(r, g["reward"][:, t], err_msg=f"t={t}")
        np.testing.assert_array_equal(d, g["done"][:, t], err_msg=f"t={t}")
        np.testing.assert_array_equal(st["agent"], g["agent"][:, t], err_msg=f"t={t}")
        np.testing.assert_array_equal(st["dist"], g["dist"][:, t], err_msg=f"t={t}")
        np.testing.assert_array_equal(st["ep_return"], g["ep_return"][:, t], err_msg=f"t={t}")
        check_features(f, g["feat"][:, t], f"t={t}")


@pytest.mark.parametrize("prefix", ["a", "b"])
def test_py_board_golden(prefix):
    """oracle/py_board.py, the scalar createBoard port timed as the board leg's CPU baseline,
    replays the reference's own episodes: the same reset draws give the same spawns, and every
    step the same reward, done, agent, distance, return and 20 features."""
    from oracle.py_board import ACTIONS, PyBoard, _Draws
    g = fixture(prefix)
    E, T = g["actions"].shape
    ns = g["init_static"].shape[1]
    for e in range(E):
        b = PyBoard(ns)
        b.reset(_Draws(g["reset_tape"][e, : int(g["reset_used"][e])]))
        assert b.state[0] == tuple(g["init_agent"][e]) and b.state[1] == tuple(g["init_goal"][e])
        assert b.state[2] == g["init_dist"][e] and b.total_distance == g["init_total"][e]
        assert [(o.x, o.y) for o in b.obstacle_list] == [tuple(p) for p in g["init_static"][e]]
        check_features(b.sensor_readings, g["init_feat"][e], f"e={e} reset")
        for t in range(T):
            state, r, d = b.step(ACTIONS[g["actions"][e, t]])
            assert r == g["reward"][e, t] and d == bool(g["done"][e, t]), (e, t)
            assert state[0] == tuple(g["agent"][e, t]) and state[2] == g["dist"][e, t], (e, t)
            assert b.total_reward_accumulated == g["ep_return"][e, t], (e, t)
            check_features(b.sensor_readings, g["feat"][e, t], f"e={e} t={t}")


def test_py_board_baseline_runs():
    from oracle import py_board
    n, el = py_board.run_baseline(0.2, seed=3)
    assert n > 0 and el > 0


def make_board(gpu, n, ns, **kw):
    from gym_ballenv_amd import BatchedBoard
    return BatchedBoard(n, ns, device=gpu, **kw)


@pytest.mark.gpu
@pytest.mark.parametrize("prefix", ["a", "b"])
def test_gpu_board_golden(gpu, prefix):
    g = fixture(prefix)
    E, T = g["actions"].shape
    ns = g["init_static"].shape[1]
    b = make_board(gpu, E, ns)
    tape = torch.from_numpy(np.ascontiguousarray(np.nan_to_num(g["reset_tape"].T[: int(g["reset_used"].max())])))
    f = b.reset(reset_tape=tape)
    b.status()
    np.testing.assert_array_equal(b.agent.cpu().numpy(), g["init_agent"])
    np.testing.assert_array_equal(b.goal.cpu().numpy(), g["init_goal"])
    np.testing.assert_array_equal(b.dist.cpu().numpy(), g["init_dist"])
    np.testing.assert_array_equal(b.total_dist.cpu().numpy(), g["init_total"])
    np.testing.assert_array_equal(b.static_obs.cpu().numpy().transpose(1, 0, 2), g["init_static"])
    check_features(f.cpu().numpy(), g["init_feat"], "reset")
    acts = torch.from_numpy(g["actions"]).to(gpu)
    for t in range(T):
        f, r, d, _ = b.step(acts[:, t])
        np.testing.assert_array_equal(r.cpu().numpy(), g["reward"][:, t], err_msg=f"t={t}")
        np.testing.assert_array_equal(d.cpu().numpy(), g["done"][:, t].astype(bool), err_msg=f"t={t}")
        np.testing.assert_array_equal(b.agent.cpu().numpy(), g["agent"][:, t], err_msg=f"t={t}")
        np.testing.assert_array_equal(b.ep_return.cpu().numpy(), g["ep_return"][:, t], err_msg=f"t={t}")
        check_features(f.cpu().numpy(), g["feat"][:, t], f"t={t}")
    b.status()
    b.close()


@pytest.mark.gpu
def test_gpu_board_philox_vs_oracle(gpu):
    """Philox resets honour the reference's spawn rules; then float-delta and index steps
    from those states are bit-exact against the oracle (N not a multiple of 256)."""
    N, ns = 5000, 8
    b = make_board(gpu, N, ns, seed=9)
    b.reset()
    b.status()
    ag, go = b.agent.cpu().numpy(), b.goal.cpu().numpy()
    so = b.static_obs.cpu().numpy().astype(np.float64)
    assert (np.hypot(*(ag - go).T) >= 50).all()
    assert ((0 <= ag) & (ag < 100)).all() and ((0 <= go) & (go < 100)).all()
    for k in range(ns):
        assert (np.sqrt(((so[k] - ag) ** 2).sum(1)) - 15 > 20).all()
        assert (np.sqrt(((so[k] - go) ** 2).sum(1)) - 5 > 20).all()
    cfg = cfg_for(N, ns)
    st = {k: getattr(b, k).cpu().numpy().copy() for k in b.STATE_KEYS}
    st["episode"] = st["episode"].view(np.uint32)
    rng = np.random.default_rng(3)
    for t in range(30):
        if t % 2:
            a = rng.integers(0, 4, N).astype(np.uint8)
            f, r, d, _ = b.step(torch.from_numpy(a))
            wr, wd, wf = oracle.board_step(cfg, st, actions=a)
        else:
            dl = rng.normal(0, 3, (N, 2))
            f, r, d, _ = b.step(deltas=torch.from_numpy(dl))
            wr, wd, wf = oracle.board_step(cfg, st, deltas=dl)
        np.testing.assert_array_equal(r.cpu().numpy(), wr, err_msg=f"t={t}")
        np.testing.assert_array_equal(d.cpu().numpy(), wd.astype(bool))
        np.testing.assert_array_equal(b.agent.cpu().numpy(), st["agent"])
        check_features(f.cpu().numpy(), wf, f"t={t}")
    b.close()


@pytest.mark.gpu
def test_gpu_board_autoreset_and_observe(gpu):
    N = 2048
    b = make_board(gpu, N, 6, seed=1, autoreset=True, time_limit=40)
    b.reset()
    ep0 = b.episode.clone()
    acts = torch.randint(0, 4, (60, N), dtype=torch.uint8, device=gpu)
    finished = torch.zeros(N, dtype=torch.bool, device=gpu)
    for t in range(60):
        _, _, d, info = b.step(acts[t])
        finished |= d
        assert bool((b.ep_len[d] == 0).all())
    assert bool(finished.all())              # every env hit, reached the goal or timed out
    assert bool((b.episode > ep0).all())
    f1 = b.features.clone()
    assert torch.equal(b.observe(), f1)      # observe() == the features step() wrote
    b.status()
    b.close()


@pytest.mark.gpu
@pytest.mark.parametrize("use_deltas", [False, True])
def test_gpu_board_rollout_matches_steps(gpu, use_deltas):
    """be_board_rollout == that many be_board_step calls, bit for bit (features, reward, done,
    truncated, state), through autoresets (wave-cooperative Philox) and a partial last block."""
    N, K = 5000, 45
    a, b = (make_board(gpu, N, 6, seed=4, autoreset=True, time_limit=20) for _ in range(2))
    a.reset()
    b.reset()
    g = torch.Generator(device="cpu").manual_seed(2)
    if use_deltas:
        mv = (torch.randn(K, N, 2, generator=g, dtype=torch.float64) * 3).to(gpu)
    else:
        mv = torch.randint(0, 4, (K, N), generator=g, dtype=torch.uint8).to(gpu)
    ref = {"f": [], "r": [], "d": [], "t": []}
    for t in range(K):
        f, r, d, info = a.step(deltas=mv[t]) if use_deltas else a.step(mv[t])
        ref["f"].append(f.clone()); ref["r"].append(r.clone()); ref["d"].append(d.clone())
        ref["t"].append(info["truncated"].clone())
    f, r, d, info = b.rollout(deltas=mv) if use_deltas else b.rollout(mv)
    assert torch.equal(f, torch.stack(ref["f"]))
    assert torch.equal(r, torch.stack(ref["r"]))
    assert torch.equal(d, torch.stack(ref["d"]))
    assert torch.equal(info["truncated"], torch.stack(ref["t"]))
    assert bool(d.any())
    for k in a.STATE_KEYS:
        assert torch.equal(getattr(a, k), getattr(b, k)), k
    a.status()
    b.status()
    a.close()
    b.close()


@pytest.mark.gpu
@pytest.mark.parametrize("ns,over", [(6, {}), (8, {}), (0, {}), (12, {}), (6, {"min_spawn_dist": 65.0}),
                                     (8, {"spawn_thresh_agent": 30.0, "spawn_thresh_goal": 25.0})])
def test_gpu_board_philox_resets_vs_oracle(gpu, ns, over):
    """Philox-mode resets (be_board_reset without a tape, and the autoreset inside be_board_step)
    bit-exact against the oracle's sequential restatement of the engine's draw layout
    (orc_board_reset_philox): a full reset, a masked reset, then 40 random moves with autoreset.
    The draws are the engine's own (Philox), so this pins the layout, not the reference.
    The single-chain pass (1 <= ns <= 12) hands envs whose rejection loops need more attempts
    than it draws to the general passes: ns = 12 (four attempts per static), a min_spawn of 65
    (the agent rejected 12 times in a row for ~9 % of resets) and wide static thresholds make those common."""
    N, seed, off = 5000, 0x5EED, 12345
    b = make_board(gpu, N, ns, seed=seed, env_offset=off, autoreset=True, **over)
    cfg = b.cfg
    st = oracle.board_new_state(cfg)
    rng = np.random.default_rng(ns)

    def check(msg):
        for k in b.STATE_KEYS:
            got = getattr(b, k).cpu().numpy()
            want = st[k].view(np.int32) if k == "episode" else st[k]
            np.testing.assert_array_equal(got, want, err_msg=f"{msg}: {k}")

    f = b.reset()
    s, wf = oracle.board_reset_philox(cfg, st)
    assert s == 0
    check("reset")
    check_features(f.cpu().numpy(), wf, "reset")
    mask = rng.random(N) < 0.3
    f = b.reset(mask=torch.from_numpy(mask))
    s, wf2 = oracle.board_reset_philox(cfg, st, mask=mask)
    check("masked reset")
    check_features(f.cpu().numpy()[mask], wf2[mask], "masked reset")
    n_done = 0
    for t in range(40):   # float mouse moves (sigma 4): hits and goals within a few dozen steps
        dl = rng.normal(0, 4, (N, 2))
        f, r, d, _ = b.step(deltas=torch.from_numpy(dl))
        wr, wd, wf = oracle.board_step(cfg, st, deltas=dl)
        dm = wd.astype(bool)
        _, wfr = oracle.board_reset_philox(cfg, st, mask=dm)
        np.testing.assert_array_equal(r.cpu().numpy(), wr, err_msg=f"reward t={t}")
        np.testing.assert_array_equal(d.cpu().numpy(), dm, err_msg=f"done t={t}")
        check(f"t={t}")
        check_features(f.cpu().numpy(), np.where(dm[:, None], wfr, wf), f"t={t}")
        n_done += int(dm.sum())
    assert n_done > N // 50, n_done
    b.status()
    b.close()


@pytest.mark.gpu
@pytest.mark.parametrize("ns", [6, 13])
def test_gpu_board_two_lanes_equal_one_lane(gpu, ns, monkeypatch):
    """The two-lanes-per-env board kernels (BALLENV_BOARD_LPE=2, an A/B option) equal the one-lane ones bit for bit:
    features (exactly, including the social-force sum, added in obstacle order), rewards, dones
    and state through Philox autoresets, for be_board_step, be_board_rollout and observe; a
    partial last block (N = 5000)."""
    N, K = 5000, 40
    boards = []
    for lpe in ("1", "2"):
        monkeypatch.setenv("BALLENV_BOARD_LPE", lpe)
        boards.append(make_board(gpu, N, ns, seed=8, autoreset=True, time_limit=25))
    monkeypatch.delenv("BALLENV_BOARD_LPE")
    for b in boards:
        b.reset()
    g = torch.Generator(device="cpu").manual_seed(ns)
    mv = torch.randint(0, 4, (2 * K, N), generator=g, dtype=torch.uint8).to(gpu)
    for t in range(K):
        res = [b.step(mv[t]) for b in boards]
        for x, y in zip(res[0][:3], res[1][:3]):
            assert torch.equal(x, y), t
    res = [b.rollout(mv[K:]) for b in boards]
    for x, y in zip(res[0][:3], res[1][:3]):
        assert torch.equal(x, y)
    assert bool(res[0][2].any())
    for k in boards[0].STATE_KEYS:
        assert torch.equal(getattr(boards[0], k), getattr(boards[1], k)), k
    assert torch.equal(boards[0].observe(), boards[1].observe())
    for b in boards:
        b.status()
        b.close()


@pytest.mark.gpu
def test_gpu_board_top_of_id_space(gpu):
    """createBoard at the top of the 32-bit global-id space (be_board_create's limit): 2^21 envs whose
    ids end at 2^32 - 1.  The last 2048 envs' Philox reset and 40 steps of float moves with autoreset
    (hits and goals; the oracle has no TimeLimit) are bit-exact against the oracle on the same global ids: state, rewards, dones,
    and the features (f[18] within 1 f32 ulp)."""
    N, ns, k = 1 << 21, 6, 2048
    off, a = (1 << 32) - N, N - k
    b = make_board(gpu, N, ns, seed=0x70B, env_offset=off, autoreset=True)
    cfg = type(b.cfg).from_buffer_copy(b.cfg)
    cfg.num_envs, cfg.env_offset = k, off + a
    st = oracle.board_new_state(cfg)

    def check(msg):
        for key in b.STATE_KEYS:
            v = getattr(b, key)
            got = (v[:, a:] if key == "static_obs" else v[a:]).cpu().numpy()
            want = st[key].view(np.int32) if key == "episode" else st[key]
            np.testing.assert_array_equal(got, want, err_msg=f"{msg}: {key}")

    f = b.reset()
    s, wf = oracle.board_reset_philox(cfg, st)
    assert s == 0
    check("reset")
    check_features(f[a:].cpu().numpy(), wf, "reset")
    g = torch.Generator(device=gpu).manual_seed(5)
    n_done = 0
    for t in range(40):
        dl = torch.randn(N, 2, generator=g, dtype=torch.float64, device=gpu) * 4
        f, r, d, _ = b.step(deltas=dl)
        wr, wd, wf = oracle.board_step(cfg, st, deltas=dl[a:].cpu().numpy())
        dm = wd.astype(bool)
        _, wfr = oracle.board_reset_philox(cfg, st, mask=dm)
        np.testing.assert_array_equal(r[a:].cpu().numpy(), wr, err_msg=f"reward t={t}")
        np.testing.assert_array_equal(d[a:].cpu().numpy(), dm, err_msg=f"done t={t}")
        check(f"t={t}")
        check_features(f[a:].cpu().numpy(), np.where(dm[:, None], wfr, wf), f"t={t}")
        n_done += int(dm.sum())
    assert n_done > k // 50, n_done
    b.status()
    b.close()


@pytest.mark.gpu
@pytest.mark.parametrize("ns,period,over", [(6, "128", {}), (13, "1", {}), (0, "3", {}), (20, "0", {}),
                                            (8, "5", {"min_spawn_dist": 65.0}), (6, "2", {"min_spawn_dist": 200.0})])
def test_gpu_board_pool_equals_inline(gpu, ns, period, over, monkeypatch):
    """The board's autoreset pool (be_board_pool_bytes > 0) changes no bit: be_board_step with the
    pool equals the inline draws (BALLENV_POOL=0) -- features, rewards, dones, truncations and state
    through autoresets, for a fill every step (period 1), a short period, the default, and no periodic
    fill (period 0: entries go stale after the first two episodes and the steps fall back to inline
    draws); general-pass envs (min_spawn 65) and an impossible spawn rule (every reset at the
    rejection limit: the REJ flag raises the status word as the inline draw does).  A masked reset
    mid-run refills the pool; a state_dict round trip (episode counters rewound) leaves the tags to
    reject what no longer matches."""
    N, K = 5000, 60
    boards = []
    for pool in ("1", "0"):
        monkeypatch.setenv("BALLENV_POOL", pool)
        monkeypatch.setenv("BALLENV_POOL_PERIOD", period)
        boards.append(make_board(gpu, N, ns, seed=21, autoreset=True, time_limit=15, **over))
    monkeypatch.delenv("BALLENV_POOL")
    monkeypatch.delenv("BALLENV_POOL_PERIOD")
    assert boards[0].pool_bytes() > 0 and boards[1].pool_bytes() == 0
    for b in boards:
        b.reset()
    snap = boards[0].state_dict()
    g = torch.Generator(device="cpu").manual_seed(ns + 1)
    mv = torch.randint(0, 4, (K, N), generator=g, dtype=torch.uint8).to(gpu)
    mask = torch.rand(N, generator=g) < 0.4
    n_done = 0
    for t in range(K):
        if t == 20:
            for b in boards:
                b.reset(mask=mask)
        if t == 40:
            for b in boards:
                b.load_state_dict(snap)
        res = [b.step(mv[t]) for b in boards]
        for x, y in zip(res[0][:3], res[1][:3]):
            assert torch.equal(x, y), t
        assert torch.equal(res[0][3]["truncated"], res[1][3]["truncated"]), t
        n_done += int(res[0][2].sum())
        for k in boards[0].STATE_KEYS:
            assert torch.equal(getattr(boards[0], k), getattr(boards[1], k)), (t, k)
    assert n_done > N
    errs = []
    for b in boards:
        try:
            b.status()
            errs.append(None)
        except Exception as e:   # the impossible spawn rule: both raise the rejection limit
            errs.append(str(e))
    assert errs[0] == errs[1]
    assert (errs[0] is not None) == (over.get("min_spawn_dist", 0) > 150), errs
    for b in boards:
        b.close()
