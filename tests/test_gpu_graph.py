"""The bench's method, checked: be_step launches captured into hipGraphs (torch.cuda.graph on a
side stream, as bench.py's graph_steps_leg does) and replayed give the same trajectory as the same
steps called eagerly -- every step's outputs, the final state and the stats slots, bit for bit --
for each fixed-shape step kernel the BASELINE configs run, and for the createBoard step."""
import ctypes as C

import numpy as np
import pytest
import torch

from test_gpu_parity import KEYS, make_env, np_state

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("W,N", [(10, 65536), (5, 4096), (10, 131072), (10, 32768)])
def test_graph_replayed_steps_equal_eager(gpu, W, N):
    from gym_ballenv_amd import _abi
    from gym_ballenv_amd.config import EnvConfig
    T, chunk = 60, 25
    cfg_py = EnvConfig(time_limit=40)   # truncations and autoresets inside the captured steps
    eager, graphed = (make_env(cfg_py, N, W, gpu, seed=123) for _ in range(2))
    acts = eager.sample_actions(T, seed=7)
    for e in (eager, graphed):
        e.reset()
    # per-step outputs of the graphed env: copied inside the graph after each step
    rec = {k: torch.empty((T,) + tuple(getattr(graphed, k).shape), dtype=getattr(graphed, k).dtype, device=gpu)
           for k in ("obs", "reward", "done", "truncated")}
    lib, ctx, st, out = graphed._lib, graphed._ctx, C.byref(graphed._st), C.byref(graphed._out)
    side = torch.cuda.Stream(gpu)
    graphs = []
    for c0 in range(0, T, chunk):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=side):
            cs = C.c_void_p(torch.cuda.current_stream(gpu).cuda_stream)
            for t in range(c0, min(T, c0 + chunk)):
                rc = lib.be_step(ctx, st, C.c_void_p(acts[t].data_ptr()), None, None, out, cs)
                if rc:
                    _abi.check(rc, ctx)
                for k, buf in rec.items():
                    buf[t].copy_(getattr(graphed, k))
        graphs.append(g)
    for g in graphs:
        g.replay()
    torch.cuda.synchronize(gpu)
    n_done = 0
    for t in range(T):
        obs, reward, done, info = eager.step(acts[t])
        n_done += int(done.sum())
        for k, v in (("obs", obs), ("reward", reward), ("done", done), ("truncated", info["truncated"])):
            assert torch.equal(rec[k][t], v), f"{k} t={t}"
    torch.cuda.synchronize(gpu)
    a, b = np_state(eager), np_state(graphed)
    for k in KEYS:
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)
    assert torch.equal(eager.stats_buf, graphed.stats_buf)
    assert n_done > 0
    assert eager.kernel_name("step") == graphed.kernel_name("step")
    for e in (eager, graphed):
        e.status()
        e.close()


def test_graph_replayed_board_steps_equal_eager(gpu):
    """The createBoard leg's method: be_board_step captured and replayed == eager steps (features,
    reward, done, truncated per step, final state), 65 536 envs, 6 statics, autoreset, a short
    TimeLimit so resets happen inside the graph."""
    from gym_ballenv_amd import BatchedBoard
    N, T = 65536, 60
    eager, graphed = (BatchedBoard(N, 6, device=gpu, seed=0xB0A2D, autoreset=True, time_limit=30) for _ in range(2))
    gen = torch.Generator(device=gpu).manual_seed(3)
    acts = torch.randint(0, 4, (T, N), dtype=torch.uint8, device=gpu, generator=gen)
    for b in (eager, graphed):
        b.reset()
    rec = {k: torch.empty((T,) + tuple(getattr(graphed, k).shape), dtype=getattr(graphed, k).dtype, device=gpu)
           for k in ("features", "reward", "done", "truncated")}
    side = torch.cuda.Stream(gpu)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=side):
        sp = C.c_void_p(torch.cuda.current_stream(gpu).cuda_stream)
        for t in range(T):
            graphed._lib.be_board_step(graphed._h, C.byref(graphed._st), C.c_void_p(acts[t].data_ptr()), None,
                                       C.byref(graphed._out), sp)
            for k, buf in rec.items():
                buf[t].copy_(getattr(graphed, k))
    g.replay()
    torch.cuda.synchronize(gpu)
    n_done = 0
    for t in range(T):
        f, r, d, info = eager.step(acts[t])
        n_done += int(d.sum())
        for k, v in (("features", f), ("reward", r), ("done", d), ("truncated", info["truncated"])):
            assert torch.equal(rec[k][t], v), f"{k} t={t}"
    for k in eager.STATE_KEYS:
        assert torch.equal(getattr(eager, k), getattr(graphed, k)), k
    assert n_done > 0
    for b in (eager, graphed):
        b.close()


def test_graph_captured_batched_step_api(gpu):
    """BatchedBallEnv.step() itself inside torch.cuda.graph: the caller's
    loop -- one torch op writing the actions into a fixed buffer, then env.step(buffer) -- captured
    and replayed equals the same loop run eagerly (step() is asynchronous on the current stream, uses
    the caller's stream handle and allocates nothing on its fast path)."""
    from gym_ballenv_amd.config import EnvConfig
    N, W, T = 32768, 10, 40
    cfg_py = EnvConfig(time_limit=25)
    eager, graphed = (make_env(cfg_py, N, W, gpu, seed=77) for _ in range(2))
    acts = eager.sample_actions(T, seed=9)
    for e in (eager, graphed):
        e.reset()
    buf = torch.empty(N, dtype=torch.uint8, device=gpu)
    graphed.step(buf.copy_(acts[0]))          # first call (checks) outside the capture; replayed below too
    rec = torch.empty((T, N, graphed.obs_dim), dtype=torch.uint8, device=gpu)
    rew = torch.empty((T, N), dtype=torch.float64, device=gpu)
    side = torch.cuda.Stream(gpu)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=side):
        for t in range(1, T):
            buf.copy_(acts[t])
            obs, reward, done, info = graphed.step(buf)
            rec[t].copy_(obs)
            rew[t].copy_(reward)
    g.replay()
    torch.cuda.synchronize(gpu)
    for t in range(T):
        obs, reward, done, info = eager.step(acts[t])
        if t:
            assert torch.equal(rec[t], obs), f"obs t={t}"
            assert torch.equal(rew[t], reward), f"reward t={t}"
    a, b = np_state(eager), np_state(graphed)
    for k in KEYS:
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)
    for e in (eager, graphed):
        e.status()
        e.close()


@pytest.mark.parametrize("W,N", [(10, 65536), (5, 4096)])
def test_short_graph_with_captured_pool_fill(gpu, W, N):
    """A graph of 8 steps plus a captured be_pool_fill, replayed 40 times (INTEGRATION.md's recipe for
    short graphs): the same trajectory as an env without the pool stepping eagerly.  TimeLimit 12, so
    every env resets several times and only the captured fills keep its entries current; the pool's
    own entries afterwards are current for the env's next two episodes (the captured fill ran)."""
    import os
    from gym_ballenv_amd import _abi
    from gym_ballenv_amd.config import EnvConfig
    K, R = 8, 40
    cfg_py = EnvConfig(time_limit=12)
    graphed = make_env(cfg_py, N, W, gpu, seed=77)
    os.environ["BALLENV_POOL"] = "0"
    try:
        eager = make_env(cfg_py, N, W, gpu, seed=77)
    finally:
        del os.environ["BALLENV_POOL"]
    assert graphed.pool_bytes() > 0 and eager.pool_bytes() == 0
    graphed.pool_set_period(0)          # no host-counted fills: only the captured one
    acts = eager.sample_actions(K, seed=9)
    for e in (eager, graphed):
        e.reset()
    lib, ctx, st, out = graphed._lib, graphed._ctx, C.byref(graphed._st), C.byref(graphed._out)
    rec = {k: torch.empty((K,) + tuple(getattr(graphed, k).shape), dtype=getattr(graphed, k).dtype, device=gpu)
           for k in ("obs", "reward", "done")}
    side = torch.cuda.Stream(gpu)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=side):
        cs = C.c_void_p(torch.cuda.current_stream(gpu).cuda_stream)
        for t in range(K):
            rc = lib.be_step(ctx, st, C.c_void_p(acts[t].data_ptr()), None, None, out, cs)
            if rc:
                _abi.check(rc, ctx)
            for k, buf in rec.items():
                buf[t].copy_(getattr(graphed, k))
        _abi.check(lib.be_pool_fill(ctx, st, cs), ctx)
    n_done = 0
    for r in range(R):
        g.replay()
        for t in range(K):
            obs, reward, done, _ = eager.step(acts[t])
            n_done += int(done.sum())
            for k, v in (("obs", obs), ("reward", reward), ("done", done)):
                assert torch.equal(rec[k][t], v), f"{k} replay {r} t={t}"
    torch.cuda.synchronize(gpu)
    a, b = np_state(eager), np_state(graphed)
    for k in KEYS:
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)
    assert n_done > 4 * N, n_done
    ep = graphed.episode.cpu().numpy().view(np.uint32)
    for i in np.random.default_rng(W).choice(N, 16, replace=False):
        for x in (int(ep[i]) + 1, int(ep[i]) + 2):
            words, _ = graphed.pool_entry(int(i), x & 1)
            assert words[0] == x and words[3] & (1 << 30), (i, x)
    for e in (eager, graphed):
        e.status()
        e.close()



@pytest.mark.parametrize("W,N", [(10, 4096), (5, 4096)])
def test_step_runs_on_the_callers_stream(gpu, W, N):
    """step() launches on the caller's current stream (the raw handle torch reports), ordered
    after the work the caller queued there: the actions are written on a side stream behind a
    ~20-ms spin, and the step on that stream must see them.  A step launched on any other stream
    would read the old actions at once and give another trajectory."""
    from gym_ballenv_amd.config import EnvConfig
    cfg_py = EnvConfig(time_limit=40)
    env, ref = (make_env(cfg_py, N, W, gpu, seed=11) for _ in range(2))
    env.reset()
    ref.reset()
    new = ref.sample_actions(3, seed=9)
    exp = []
    for t in range(3):
        exp.append([x.clone() for x in ref.step(new[t], copy=True)[:3]])
    acts = torch.full((N,), 5, dtype=torch.uint8, device=gpu)   # action 5 = (0, 0): another trajectory
    torch.cuda.synchronize(gpu)
    side = torch.cuda.Stream(gpu)
    got = []
    with torch.cuda.stream(side):
        for t in range(3):
            torch.cuda._sleep(50_000_000)
            acts.copy_(new[t])
            got.append([x.clone() for x in env.step(acts)[:3]])
    side.synchronize()
    for t in range(3):
        for k, (a, b) in enumerate(zip(exp[t], got[t])):
            assert torch.equal(a, b), (t, ("obs", "reward", "done")[k])
    for k in KEYS:
        assert torch.equal(getattr(env, k), getattr(ref, k)), k
    # the check has teeth: the same calls with step() sent to the default stream instead read the
    # actions before the side stream writes them
    wrong = make_env(cfg_py, N, W, gpu, seed=11)
    wrong.reset()
    wrong._stream_int = lambda: torch.cuda.default_stream(gpu).cuda_stream
    acts2 = torch.full((N,), 5, dtype=torch.uint8, device=gpu)
    torch.cuda.synchronize(gpu)
    with torch.cuda.stream(side):
        torch.cuda._sleep(50_000_000)
        acts2.copy_(new[0])
        wrong.step(acts2)
    torch.cuda.synchronize(gpu)
    assert not torch.equal(wrong.reward, exp[0][1])
    for e in (env, ref, wrong):
        e.close()
