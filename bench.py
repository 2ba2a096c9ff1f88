#!/usr/bin/env python3
"""Throughput benchmark of the batched BallEnv step (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--envs E] [--window 10]
    (N > 1: torchrun --nproc-per-node N ... bench.py --gpus N, one rank per GPU)

A "step" = one be_step launch over the whole local batch: agent move, obstacle
moves (Philox), collision, reward/done, TimeLimit(1000), in-kernel autoreset and
the W x W prep_state4 window obs, for every env (ballenv_env.py:232-289 +
ball_cnn_ac3.py:384-412).  Actions are uniform random indices (the
random-action rollout of BASELINE configs 2-4), pre-generated in HBM with
be_sample_actions before the timed region; obstacle draws are Philox.
Per GPU: --envs envs (default 65536 = config 3, weak scaling across ranks);
every global env has the same trajectory at any GPU count.

Timed region: the K steps replayed from HIP graphs of captured be_step
launches (Philox draws are keyed by per-env state -- env id, episode,
ep_len -- so replays are fresh steps), bracketed by barrier + synchronize,
max over ranks.
Kernel duration for the roofline: HIP events recorded on the replay stream
around the timed region (K back-to-back be_kernel launches, nothing else on the
stream) -> average per launch; it includes the small inter-launch gap, so it is
an upper bound on the kernel duration that rocprofv3 reports.
CPU baseline (rank 0, N=1 only, before any GPU work): oracle/py_ballenv.py,
the reference's algorithm restated in scalar Python, one process per core.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
DIST_ON = False         # a torch.distributed process group is up (any launch under torchrun, even 1 rank)
LAST_OWN_ELAPSED = 0.0  # timed_graph_steps: this rank's own wall time of its last timed region


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=1000)
    p.add_argument("--warmup", type=int, default=100)
    p.add_argument("--envs", type=int, default=65536, help="envs per GPU")
    p.add_argument("--window", type=int, default=10)
    p.add_argument("--mode", choices=["loop", "graph", "eager"], default="graph",
                   help="loop: be_step_n, the K step launches queued by the library's C loop; graph: "
                        "hipGraph replay of captured be_step launches; eager: one ctypes be_step call per step")
    p.add_argument("--cpu-seconds", type=float, default=12.0)
    p.add_argument("--cpu-procs", type=int, default=0, help="0 = one per usable host core")
    p.add_argument("--board-cpu-seconds", type=float, default=6.0,
                   help="createBoard CPU baseline (oracle/py_board.py on every host core) beside the board leg "
                        "(0 = skip)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--graph-chunk", type=int, default=250, help="steps per captured graph")
    p.add_argument("--settle", type=int, default=400,
                   help="untimed steps since reset before the timed region (at least --warmup + one pass of the "
                        "K timed steps; more untimed passes until this many)")
    p.add_argument("--policy-steps", type=int, default=1000,
                   help="config 5 leg: timed steps of the on-GPU policy rollout (0 = skip)")
    p.add_argument("--torch-policy-steps", type=int, default=50,
                   help="config 5 comparison: timed steps with the PyTorch-ROCm policy (0 = skip)")
    p.add_argument("--cold-steps", type=int, default=2000,
                   help="steps of the cold-action-rows line (a fresh tape read from HBM; 0 = skip)")
    p.add_argument("--rollout-steps", type=int, default=1000,
                   help="fused be_rollout leg (SURVEY 8(d) fused multi-step mode): timed steps (0 = skip)")
    p.add_argument("--rollout-chunk", type=int, default=100, help="steps per be_rollout launch")
    p.add_argument("--dist-backend", choices=["nccl", "gloo"], default="nccl",
                   help="N > 1 collective backend (nccl = RCCL over xGMI); gloo only to rehearse the "
                        "multi-rank path with several ranks sharing one GPU")
    p.add_argument("--board-steps", type=int, default=1000,
                   help="createBoard profile leg (SURVEY 8(f) rank 2): timed steps (0 = skip)")
    p.add_argument("--config2-steps", type=int, default=1000,
                   help="BASELINE config 2 leg (4096 envs/GPU, W=5, step API): timed steps (0 = skip)")
    p.add_argument("--config2-envs", type=int, default=4096)
    p.add_argument("--config4-steps", type=int, default=1000,
                   help="BASELINE config 4 leg (a fixed 262144-env batch at W=10 split over the ranks, strong "
                        "scaling): timed steps (0 = skip)")
    p.add_argument("--config4-envs", type=int, default=262144, help="config 4: global envs over all ranks")
    p.add_argument("--large-steps", type=int, default=200,
                   help="large-batch leg (2^20 envs/GPU, W=10: past the 256-MB Infinity Cache): timed steps "
                        "(0 = skip)")
    p.add_argument("--large-envs", type=int, default=1 << 20)
    p.add_argument("--blocks-launches", type=int, default=200,
                   help="prep_state2 block-count leg (SURVEY 8(f) rank 3, be_observe_blocks): timed launches "
                        "at --envs and at --large-envs (0 = skip)")
    p.add_argument("--from-reset-steps", type=int, default=400,
                   help="the headline step timed straight from a fresh reset (no settle): timed steps (0 = skip)")
    p.add_argument("--shard-steps", type=int, default=1000,
                   help="config 4's per-rank shards (131072 / 65536 / 32768 envs = the N = 2 / 4 / 8 split) timed on "
                        "one GPU, N = 1 only: timed steps per shard (0 = skip)")
    p.add_argument("--eager-steps", type=int, default=1000,
                   help="the drop-in as its caller drives it: BatchedBallEnv.step(actions) called from Python per "
                        "step, no graph (examples/ball_cnn_ac3.py:588 for every env): timed calls (0 = skip)")
    return p.parse_args()


def launch_ranks(args):
    """`bench.py --gpus N` (N > 1) run outside torch.distributed.run: start
    `python -m torch.distributed.run --nproc-per-node N bench.py ...` as a CHILD process (never an
    exec; nothing here has touched a GPU), relay its output (rank 0 prints the JSON line) and
    return its exit code.  The driver's own form (torchrun ... bench.py --gpus N) sets WORLD_SIZE
    and never comes here."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *sys.argv[1:]]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    env.setdefault("OMP_NUM_THREADS", "1")
    print(f"bench: launching {args.gpus} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
    p = subprocess.Popen(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, text=True)
    for line in p.stdout:
        sys.stdout.write(line)
        sys.stdout.flush()
    return p.wait()


def host_cores():
    """CPUs this process may actually use: the affinity mask, capped by a cgroup-v2 CPU quota
    (on a shared GPU box os.cpu_count() and the affinity mask show the whole machine)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            n = min(n, max(1, -(-int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return max(1, n)


def cpu_baseline(window, seconds, procs=None):
    """Reference algorithm (scalar Python port of BallEnv.step + prep_state4, oracle/py_ballenv.py)
    on the host cores, SURVEY.md 8(d): single env per process, one process per usable core, at
    W=5 and W=10 (per-core and aggregate rates), plus BASELINE config 1 (one single-env W=5
    100-step rollout).  No GPU is touched.  `value` is the headline window's aggregate."""
    from oracle import py_ballenv
    import multiprocessing as mp
    cores = host_cores() if not procs else min(procs, host_cores())
    ctx = mp.get_context("fork")
    by_w = {}
    per_w = seconds / 2.0
    with ctx.Pool(cores) as pool:
        for w in (5, 10):
            res = pool.map(py_ballenv._worker, [(w, per_w, 1000 + i) for i in range(cores)])
            steps = sum(s for s, _ in res)
            el = max(t for _, t in res)
            rates = [s / t for s, t in res]
            by_w[w] = {"aggregate": steps / el, "per_core_mean": sum(rates) / len(rates),
                       "per_core_min": min(rates), "per_core_max": max(rates), "env_steps": steps,
                       "seconds": el}
    n1, t1 = py_ballenv.run_rollout(5, 100, seed=7)
    hw = by_w.get(window, by_w[10])
    return {"value": hw["aggregate"], "unit": "env-steps/s", "cores": cores, "kind": "port",
            "per_core": hw["per_core_mean"],
            "by_window": {f"W={w}": v for w, v in by_w.items()},
            "config1": {"what": "BASELINE config 1: single env, W=5, one 100-step random-action rollout, 1 core",
                        "seconds": t1, "env_steps_per_s": n1 / t1},
            "sample": f"{cores} procs (one per usable core: affinity mask, cgroup quota) x {per_w:.0f} s at W=5 "
                      f"and at W=10: single-env BallEnv.step + prep_state4, 13 static + 5 dynamic obstacles, "
                      f"uniform random 9-way actions, reset on done/1000 steps (oracle/py_ballenv.py, pure "
                      f"Python); value = W={window if window in by_w else 10} aggregate"}


def board_cpu_baseline(seconds, procs=None, static_obstacles=6):
    """The createBoard profile on the host cores (north_star's "reference single-env
    pygame step() timed on the box's own host cores"): oracle/py_board.py, the scalar port of
    createBoard.step + featureExtractor (ballenv_pygame.py:650-706, featureExtractor.py:247-265),
    single env per process, one process per usable core, random actionArray moves, reset on
    done / 1000 steps -- the board leg's workload (6 statics).  Checked within +-25 % of the
    reference's own speed in the build container (tools/cpu_port_speed.py,
    profiles/r04_cpu_port_speed.json).  No GPU is touched."""
    from oracle import py_board
    import multiprocessing as mp
    cores = host_cores() if not procs else min(procs, host_cores())
    with mp.get_context("fork").Pool(cores) as pool:
        res = pool.map(py_board._worker, [(seconds, 2000 + i, static_obstacles) for i in range(cores)])
    steps = sum(s for s, _ in res)
    el = max(t for _, t in res)
    rates = [s / t for s, t in res]
    return {"value": steps / el, "unit": "env-steps/s", "cores": cores, "kind": "port",
            "per_core": sum(rates) / len(rates), "per_core_min": min(rates), "per_core_max": max(rates),
            "env_steps": steps, "seconds": el,
            "sample": f"{cores} procs (one per usable core) x {seconds:.0f} s: single-env createBoard.step + "
                      f"featureExtractor, {static_obstacles} static obstacles, random actionArray moves, reset on "
                      "done / 1000 steps (oracle/py_board.py, pure Python + numpy)"}


def gb_step_bytes(env):
    """be_step_bytes of an env's config: the bytes the engine's layout moves per env-step."""
    import gym_ballenv_amd as gb
    return gb.step_bytes(env.cfg, env.window)


def timed_graph_steps(graphs, steps, dev, stream, world):
    """Replay graphs (steps in total), bracketed by barrier + synchronize; max over ranks."""
    import torch
    import torch.distributed as dist
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if DIST_ON:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ev0.record(stream)
    t0 = time.perf_counter()
    for g in graphs:
        g.replay()
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    global LAST_OWN_ELAPSED
    LAST_OWN_ELAPSED = el       # this rank's own wall time (the per-rank rows of graph_steps_leg)
    if DIST_ON:
        dist.barrier()
    if DIST_ON:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    return el, ev0.elapsed_time(ev1) / steps


def pool_info(env):
    """The autoreset pool of an env's context (include/ballenv.h): every step launch of the timed
    region is the step kernel plus, every `period` launches, one pool_fill_kernel launch -- the event
    time per step (kernel_us_mean) includes the fills; a rocprof trace splits the two
    (tools/trace_regions.py)."""
    b = env.pool_bytes()
    if not b:
        return None
    p = env.pool_period()
    return {"bytes": b, "period": p, "fill_kernel": f"pool_fill_kernel<{env.window}, 13, 5>",
            "fills_per_step": (1.0 / p) if p else 0.0,
            "note": "kernel_us_mean (HIP events over the timed region) covers the step launches and the "
                    "fill launches between them"}


def rank_rows(dev, row):
    """Per-rank diagnostics of a timed region at N > 1 (the row of every rank, all_gather_object):
    a scaling run then explains its own curve -- which rank / GPU was slow, by how much, and what
    the stats exchange cost."""
    import torch
    import torch.distributed as dist
    row = dict(row, rank=dist.get_rank(), host=os.uname().nodename,
               device_uuid=str(torch.cuda.get_device_properties(dev).uuid))
    rows = [None] * dist.get_world_size()
    dist.all_gather_object(rows, row)
    return rows


def cold_actions_leg(args, env, lib, dev, stream, world, B):
    """The headline step on action rows that come from HBM.  The headline's K rows are replayed by
    the untimed settle pass first, so they sit in the Infinity Cache -- as actions a policy writes
    just before each step do.  Here: a fresh (steps, N) tape that no step has read, and a 512-MB
    write before the timed pass evicts the caches, so every step's 64-KB row is an HBM miss."""
    import ctypes as C
    import torch
    T, N, chunk = args.cold_steps, env.num_envs, 250
    tape = env.sample_actions(T, seed=0xC01D)
    st_ref, out_ref = C.byref(env._st), C.byref(env._out)
    graphs = []
    cap = torch.cuda.Stream(dev)
    for c0 in range(0, T, chunk):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=cap):
            cs = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
            for t in range(c0, min(T, c0 + chunk)):
                rc = lib.be_step(env._ctx, st_ref, C.c_void_p(tape[t].data_ptr()), None, None, out_ref, cs)
                if rc:
                    raise RuntimeError(f"be_step: {rc}")
        graphs.append(g)
    flush = torch.empty(512 << 20, dtype=torch.uint8, device=dev)
    flush.fill_(1)
    el, ms = timed_graph_steps(graphs, T, dev, stream, world)
    del graphs, flush
    env.status()
    res = {"what": f"the headline step, {T} steps on a fresh action tape read from HBM (caches flushed by a "
                   "512-MB write before the timed pass); the headline's rows are Infinity-Cache resident",
           "value": T * N * world / el, "unit": "env-steps/s", "ms_per_step": el / T * 1e3,
           "kernel_us_mean": ms * 1e3, "frac": B * N / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS}
    return moved(res, gb_step_bytes(env), N, ms * 1e3, None)


def policy_leg(args, gb, dev, rank, world, stream):
    """BASELINE config 5: the same env batch driven by the reference's Policy(W) on the GPU.

    Reported: the fused rollout (be_policy_rollout, one kernel per chunk of steps) with the
    two-launch loop below and the PyTorch-ROCm policy as comparison points (same trajectory
    for the two HIP paths, tests/test_gpu_rollout.py).

    One step = be_policy_act (select_action, csrc/policy.hip) + be_step, both
    writing into (T, N) trajectory rows, captured in HIP graphs.  The policy is
    the reference's trained Policy(W) (tests/golden/policy_w{W}.npz) when the
    fixture exists, else a random-init Policy(W).
    """
    import torch
    from gym_ballenv_amd.policy import HipPolicy, Policy, reference_weights
    N, W, T = args.envs, args.window, args.policy_steps
    path = reference_weights(W)
    torch.manual_seed(0)
    pol = Policy.from_npz(path, W) if path else Policy(W)
    res = {"workload": f"config 5: Policy({W}) select_action (be_policy_act, int8-MFMA fc1) + be_step, "
                       f"{N} envs/GPU, T={T} steps per rollout, hipGraph replay (two launches per step)",
           "weights": os.path.relpath(path, ROOT) if path else "random init"}
    env = gb.BatchedBallEnv(N, W, gb.EnvConfig(), device=dev, seed=0xBA11, env_offset=rank * N)
    env.reset()
    ro = gb.Rollout(env, pol, horizon=T, backend="hip", seed=0x5E1EC7)
    ro.run_eager()                                   # warm-up rollout
    ro.capture(chunk=min(T, 100))
    ro.run()
    el, ms = timed_graph_steps(ro._graphs, T, dev, stream, world)
    res.update({"value": T * N * world / el, "unit": "env-steps/s", "ms_per_step": el / T * 1e3,
                "gpu_us_per_step": ms * 1e3})
    # the policy kernel alone (same stream, graph of T launches)
    hp = ro.hp
    g = torch.cuda.CUDAGraph()
    cap = torch.cuda.Stream(dev)
    import ctypes as C
    with torch.cuda.graph(g, stream=cap):
        sp = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        for _ in range(T):
            hp._lib.be_policy_act(hp._h, C.byref(env._st), env.obs.data_ptr(), C.byref(ro._act_outs[0]), 7, sp)
    g.replay()
    _, pms = timed_graph_steps([g], T, dev, stream, world)
    res.update({"policy_kernel_us": pms * 1e3, "packed_weight_bytes": hp.packed_bytes})
    episodes = env.episode_stats()
    res["episodes"] = {k: episodes[k] for k in ("episodes", "mean_return", "mean_length")}
    del g
    ro.close()
    env.close()
    # the same rollout fused: be_policy_rollout, select_action + step in one kernel per chunk
    env = gb.BatchedBallEnv(N, W, gb.EnvConfig(), device=dev, seed=0xBA11, env_offset=rank * N)
    env.reset()
    ro = gb.Rollout(env, pol, horizon=T, backend="fused", seed=0x5E1EC7, chunk=args.rollout_chunk)
    ro_chunk, img_bytes = ro.chunk, ro.hp.packed_bytes
    ro.run()                                         # warm-up horizon
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if DIST_ON:
        import torch.distributed as dist
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    ev0.record(stream)
    ro.run()
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    if DIST_ON:
        dist.barrier()
    el = time.perf_counter() - t0
    if DIST_ON:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    fused = {"workload": f"config 5: Policy({W}) select_action + be_step of {N} envs/GPU in one kernel "
                         f"(be_policy_rollout, {ro.chunk} steps per launch, packed policy in LDS, state in "
                         f"registers), T={T} steps; trajectory bit-identical to the two-launch loop",
             "weights": res["weights"], "value": T * N * world / el, "unit": "env-steps/s",
             "ms_per_step": el / T * 1e3, "kernel_us_per_step": ev0.elapsed_time(ev1) * 1e3 / T}
    episodes = env.episode_stats()
    fused["episodes"] = {k: episodes[k] for k in ("episodes", "mean_return", "mean_length")}
    env.status()
    ro.close()
    env.close()
    if args.torch_policy_steps > 0:
        Tt = args.torch_policy_steps
        env = gb.BatchedBallEnv(N, W, gb.EnvConfig(), device=dev, seed=0xBA11, env_offset=rank * N)
        env.reset()
        ro = gb.Rollout(env, pol, horizon=Tt, backend="torch")
        ro.run_eager()
        ro.capture(chunk=Tt)
        ro.run()
        el_t, _ = timed_graph_steps(ro._graphs, Tt, dev, stream, world)
        fused["torch_policy"] = {"value": Tt * N * world / el_t, "unit": "env-steps/s", "ms_per_step": el_t / Tt * 1e3,
                                 "what": "same loop with select_action in PyTorch-ROCm fp32 (Linear/softmax/cumsum "
                                         "draw), hipGraph replay"}
        ro.close()
        env.close()
    fused["two_launch"] = res
    fused["roofline"] = policy_roofline(args, gb, dev, rank, pol, fused["kernel_us_per_step"], ro_chunk, img_bytes)
    return fused


def policy_roofline(args, gb, dev, rank, pol, us_per_step, chunk, img):
    """Roofline of the fused config-5 kernel on what it actually issues.

    fc1 runs on the int8 matrix cores only for envs whose window has a lit cell: each
    workgroup (256 envs) packs those into 16-env tiles, and each tile costs HT x KS x 3
    v_mfma_i32_16x16x64_i8 (hidden-row tiles x K-steps x 3 digit planes, csrc/policy_core.h).
    The envs with an empty window read their logits from a 4-entry table (no MFMA).  The tile
    count per step is measured on a recorded rollout of the same env batch and policy (the
    policy input obs of every step), so `achieved` counts MFMA ops issued, not 2*N*F*H."""
    import torch
    from gym_ballenv_amd.rollout import Rollout
    N, W, T = args.envs, args.window, 100
    env = gb.BatchedBallEnv(N, W, gb.EnvConfig(), device=dev, seed=0xBA11, env_offset=rank * N)
    env.reset()
    ro = Rollout(env, pol, horizon=T, backend="fused", record_obs=True, seed=0x5E1EC7, chunk=T)
    ro.run()
    lit = (ro.obs[:T, :, 4:] != 0).any(-1).to(torch.int32)             # (T, N): policy input has a lit cell
    nb = (N + 255) // 256
    per_block = torch.nn.functional.pad(lit, (0, nb * 256 - N)).view(T, nb, 256).sum(-1)
    tiles = (per_block + 15) // 16
    tiles_per_step = float(tiles.sum()) / T
    lit_frac = float(lit.sum()) / (T * N)
    ro.close()
    env.close()
    F = 4 + W * W
    HT, KS = -(-pol.hidden_layer // 16), -(-F // 64)
    mfma_per_tile = HT * KS * 3
    ops_step = tiles_per_step * mfma_per_tile * 2 * 16 * 16 * 64
    achieved = ops_step / (us_per_step * 1e-6) / 1e12
    peak = 5000.0      # dense int8 MFMA TOP/s (2x the ~2.5 PFLOP/s dense bf16 rate, MI355X_MICROARCH.md)
    # HBM bytes per env-step: action 1 + log_prob 4 + value 4 + reward 8 + done 1 per step, the engine
    # state read+write (161 B at the defaults) and the packed policy image (per workgroup) once per launch
    B_state = gb.step_bytes(gb.EnvConfig(), W) - (1 + 8 + 1 + 4 + W * W)
    B = 18 + B_state / chunk + (img * nb) / (chunk * N)
    res = {"bound": "mfma", "achieved": achieved, "peak": peak, "unit": "TOP/s", "frac": achieved / peak,
           "traffic": None, "tiles_per_step": tiles_per_step, "lit_env_frac": lit_frac,
           "mfma_per_tile": mfma_per_tile, "int8_ops_issued_per_step": ops_step,
           "hbm_bytes_per_env_step": B, "hbm_GBs": B * N / (us_per_step * 1e-6) / 1e9,
           "hbm_frac": B * N / (us_per_step * 1e-6) / 1e9 / HBM_PEAK_GBS,
           "limiter": "neither roofline: VALU-issue/latency-bound at one wave per SIMD (65536 envs in 256-thread "
                      "blocks are one block per CU, and the 89-KB policy image leaves LDS for only one): env "
                      "physics, select_action's softmax/draw and the head FMAs of the dense tiles"}
    # counters of the same kernel / envs / chunk (tools/pmc_passes.sh + tools/pmc_report.py, committed profile)
    d = newest_pmc("pmc_policy_rollout.json", f"rollout_kernel<{W}, 13, 5, {HT}, {KS},", N * chunk)
    if d:
        res.update({"traffic": d["hbm_bytes_per_dispatch"], "traffic_unit": f"HBM bytes per launch ({chunk} steps)",
                    "traffic_per_env_step": d["hbm_bytes_per_unit"],
                    "valu_active_frac": d.get("valu_active_per_simd_frac_est"),
                    "mfma_busy_frac": d.get("mfma_busy_frac_est"),
                    "lds_bank_conflict_frac": d.get("lds_bank_conflict_frac"),
                    "wave_cycle_split": d.get("wave_cycle_split"),
                    "pmc_source": d["source"]})
    b = d["hbm_bytes_per_dispatch"] if d else B * N * chunk     # bytes one launch (chunk steps) moves
    res.update({"moved_bytes_per_launch": b, "moved_source": d["source"] if d else "algorithmic (above)",
                "moved_frac": b / (us_per_step * chunk * 1e-6) / 1e9 / HBM_PEAK_GBS})
    return res


def rollout_leg(args, gb, dev, rank, world, stream, N=None, W=None, env_offset=None,
                pmc_suffix="pmc_rollout_kernel.json", label=None):
    """SURVEY 8(d) fused multi-step mode: the same random-action rollout as the headline, but
    be_rollout runs --rollout-chunk steps per launch with each env's state in registers
    (bit-identical outputs to be_step, tests/test_gpu_rollout.py).  Per step it writes the
    obs row, reward, done and truncated of every env into (K, N, ...) trajectory buffers.
    N / W / env_offset: another BASELINE size of the same mode (config 2's 4 096 envs at W=5:
    rolloutw_kernel; config 4's 32 768-env shard at the last rank's ids); pmc_suffix names its
    committed counter profile (profiles/rNN_<suffix>)."""
    import ctypes as C
    import torch
    from gym_ballenv_amd import _abi
    N = args.envs if N is None else N
    W = args.window if W is None else W
    T, Kc = args.rollout_steps, max(1, min(args.rollout_chunk, args.rollout_steps))
    T -= T % Kc
    off = rank * N if env_offset is None else env_offset
    env = gb.BatchedBallEnv(N, W, gb.EnvConfig(), device=dev, seed=0xBA11, env_offset=off)
    acts = env.sample_actions(T, seed=0xBA11)
    env.reset()
    env.rollout(acts[:Kc])                    # warm-up launch; allocates the (Kc, N, ...) buffers
    obs, rew, done, info = env.rollout(acts[:Kc])
    out = _abi.BeOut(obs.data_ptr(), None, rew.data_ptr(), done.data_ptr(), info["truncated"].data_ptr(), None,
                     info["final_return"].data_ptr(), info["final_len"].data_ptr(), env.stats_buf.data_ptr())
    lib, ctx, st = env._lib, env._ctx, C.byref(env._st)
    a0 = acts.data_ptr()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    sp = C.c_void_p(stream.cuda_stream)
    if DIST_ON:
        import torch.distributed as dist
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    ev0.record(stream)
    for c0 in range(0, T, Kc):
        rc = lib.be_rollout(ctx, st, C.c_void_p(a0 + c0 * N), Kc, C.byref(out), sp)
        if rc:
            _abi.check(rc, ctx)
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    if DIST_ON:
        dist.barrier()
    el = time.perf_counter() - t0
    if DIST_ON:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    us_step = ev0.elapsed_time(ev1) * 1e3 / T
    env.status()
    # algorithmic bytes / env-step (SURVEY 8(d) fused mode): action 1 + reward 8 + done 1 + truncated 1
    # + obs (4+W^2), plus the engine's state read+write (275 - 115 = 161 B at the defaults) once per launch
    B_io = 1 + 8 + 1 + 1 + 4 + W * W
    B_state = gb.step_bytes(gb.EnvConfig(), W) - (1 + 8 + 1 + 4 + W * W)
    B = B_io + B_state / Kc
    res = {"workload": (label or f"random-action rollout, {N} envs/GPU, W={W}") +
                       f", be_rollout {Kc} steps per launch "
                       "(state in registers; per-step obs/reward/done/truncated to (K, N, ...) buffers)",
           "envs": N, "window": W, "env_offset": off, "steps_per_launch": Kc,
           "value": T * N * world / el, "unit": "env-steps/s", "ms_per_step": el / T * 1e3,
           "kernel_us_per_step": us_step, "bytes_per_env_step": B,
           "achieved_GBs": B * N / (us_step * 1e-6) / 1e9,
           "frac": B * N / (us_step * 1e-6) / 1e9 / HBM_PEAK_GBS}
    # HBM-side bytes per env-step of the same kernel / envs / chunk (committed PMC passes, used only
    # when they were taken on the kernel this run launched)
    kname = env.kernel_name("rollout")
    res["kernel"] = kname
    d = newest_pmc(pmc_suffix, f"::{kname}(", N * Kc)
    if d:
        res.update({"traffic_per_env_step": d["hbm_bytes_per_unit"], "traffic_source": d["source"],
                    "measured_frac": d["hbm_bytes_per_dispatch"] / (us_step * Kc * 1e-6) / 1e9 / HBM_PEAK_GBS})
    moved(res, B, N * Kc, us_step * Kc, d, "algorithmic (above)")
    env.close()
    return res


def graph_steps_leg(gb, dev, rank, world, stream, N, W, T, settle, seed=0xBA11, chunk=250, env_offset=None,
                    global_envs=None):
    """be_step of N envs/GPU at window W, T steps replayed from hipGraphs of captured launches
    (the headline's method), after `settle` untimed steps since reset (0: timed straight from
    the reset).  Envs are the global ids [env_offset, env_offset + N) (default rank * N: weak
    scaling); `global_envs` (strong scaling: a fixed batch split over the ranks) sets the
    env-steps counted per step and adds the ranks' combined episode statistics (all_gather) of
    the TIMED steps (the statistics slots are zeroed after the untimed settle replays).
    Returns (result dict, kernel name); the env is closed."""
    import ctypes as C
    import torch
    from gym_ballenv_amd import _abi
    cfg = gb.EnvConfig()
    off = rank * N if env_offset is None else env_offset
    env = gb.BatchedBallEnv(N, W, cfg, device=dev, seed=seed, env_offset=off)
    acts = env.sample_actions(T, seed=seed)
    lib, ctx, st, out = env._lib, env._ctx, C.byref(env._st), C.byref(env._out)
    graphs, cap = [], torch.cuda.Stream(dev)
    env.reset()
    for c0 in range(0, T, chunk):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=cap):
            cs = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
            for t in range(c0, min(T, c0 + chunk)):
                rc = lib.be_step(ctx, st, C.c_void_p(acts[t].data_ptr()), None, None, out, cs)
                if rc:
                    _abi.check(rc, ctx)
        graphs.append(g)
    untimed = 0
    while True:          # the first replay uploads the graphs; then settle (or reset again)
        for g in graphs:
            g.replay()
        untimed += T
        if untimed >= max(settle, 1):
            break
    if settle <= 0:
        env.reset()      # timed straight from a fresh reset (in place: the graphs' buffers)
        untimed = 0
    env.clear_stats()    # in place (the graphs' stats pointer): episodes of the timed steps only
    torch.cuda.synchronize(dev)
    el, ms = timed_graph_steps(graphs, T, dev, stream, world)
    own_el = LAST_OWN_ELAPSED
    env.status()
    kname = env.kernel_name("step")
    pool = pool_info(env)
    episodes = rows = None
    if global_envs is not None:
        t_ag = time.perf_counter()
        per_rank = gb.gather_stats(env.stats_record()) if DIST_ON else env.stats_record().reshape(1, -1)
        torch.cuda.synchronize(dev)
        ag_us = (time.perf_counter() - t_ag) * 1e6
        episodes = gb.combine_stats(per_rank)
        if DIST_ON and world > 1:
            rows = rank_rows(dev, {"envs": N, "env_offset": off, "kernel": kname, "kernel_us_mean": ms * 1e3,
                                   "ms_per_step": own_el / T * 1e3, "stats_all_gather_us": ag_us})
    del graphs
    env.close()
    B = gb.survey_step_bytes(cfg, W)
    B_eng = gb.step_bytes(cfg, W)
    us = ms * 1e3
    units = N * world if global_envs is None else global_envs
    res = {"value": T * units / el, "unit": "env-steps/s", "ms_per_step": el / T * 1e3, "steps": T,
           "untimed_steps_since_reset": untimed, "envs_per_gpu": N, "window": W, "kernel": kname,
           "kernel_us_mean": us,
           "roofline": {"bound": "hbm", "bytes_per_env_step": B, "achieved": B * N / (us * 1e-6) / 1e9,
                        "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": B * N / (us * 1e-6) / 1e9 / HBM_PEAK_GBS,
                        "engine_bytes_per_env_step": B_eng,
                        "engine_frac": B_eng * N / (us * 1e-6) / 1e9 / HBM_PEAK_GBS, "traffic": None,
                        "measured_frac": None}}
    moved(res["roofline"], B_eng, N, us, None)    # legs with a committed profile re-run it (add_measured)
    if episodes is not None:
        res["episodes"] = episodes
    if rows is not None:
        res["per_rank"] = rows
    if pool:
        res["autoreset_pool"] = pool
    return res, kname


def add_measured(rf, pmc, us, units):
    """roofline.traffic / measured_frac from the newest committed PMC profile (bytes per launch), and
    moved_frac (PMC bytes, else the engine's be_step_bytes)."""
    if pmc:
        t = pmc["hbm_bytes_per_dispatch"]
        rf.update({"traffic": t, "measured_GBs": t / (us * 1e-6) / 1e9,
                   "measured_frac": t / (us * 1e-6) / 1e9 / HBM_PEAK_GBS, "traffic_source": pmc["source"]})
    return moved(rf, rf["engine_bytes_per_env_step"], units, us, pmc)


def eager_step_leg(args, gb, dev, rank, world, stream, graph_kernel_us):
    """The drop-in as its caller drives it (examples/ball_cnn_ac3.py:553-613, env.step at :588, for
    every env): BatchedBallEnv.step(actions) called from Python once per step, no graph; each step's
    actions come from one torch op (random_ into a preallocated (N,) u8 buffer), as a policy's
    output would.  Reported: host microseconds per step() call (the Python + ctypes + HIP launch
    cost of the call itself), host microseconds per loop iteration (the action op included), GPU
    microseconds per iteration (events around the loop: the action op's kernel + be_step + gaps),
    and env-steps/s of the whole loop beside the graph-replayed headline kernel time."""
    import torch
    N, W, T = args.envs, args.window, args.eager_steps
    env = gb.BatchedBallEnv(N, W, gb.EnvConfig(), device=dev, seed=0xBA11, env_offset=rank * N)
    env.reset()
    acts = torch.empty(N, dtype=torch.uint8, device=dev)
    for _ in range(max(args.settle, 50)):           # untimed: past the post-reset transient, caches warm
        acts.random_(0, 9)
        env.step(acts)
    env.status()
    call = 0.0
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if DIST_ON:
        import torch.distributed as dist
        dist.barrier()
    torch.cuda.synchronize(dev)
    pc = time.perf_counter
    ev0.record(stream)
    t0 = pc()
    for _ in range(T):
        acts.random_(0, 9)
        c0 = pc()
        env.step(acts)
        call += pc() - c0
    t_issue = pc() - t0
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    el = pc() - t0
    if DIST_ON:
        dist.barrier()
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    env.status()
    gpu_us = ev0.elapsed_time(ev1) * 1e3 / T
    res = {"workload": f"BatchedBallEnv.step(actions) from Python, {N} envs/GPU, W={W}, one call per step (no "
                       "graph), actions from acts.random_(0, 9) into a preallocated u8 buffer each step",
           "value": T * N * world / el, "unit": "env-steps/s", "ms_per_step": el / T * 1e3, "steps": T,
           "host_us_per_step_call": call / T * 1e6, "host_us_per_iteration": t_issue / T * 1e6,
           "gpu_us_per_iteration": gpu_us, "graph_replayed_step_kernel_us": graph_kernel_us,
           "kernel": env.kernel_name("step"),
           "host_call_over_kernel": (call / T * 1e6) / graph_kernel_us,
           "bound": "host (the GPU waits on the calls)" if t_issue / T * 1e6 >= 0.9 * gpu_us else "gpu"}
    env.close()
    return res


def config2_leg(args, gb, dev, rank, world, stream):
    """BASELINE config 2: 4096 envs/GPU at W=5, random actions, the step API (one be_step launch
    per step, graph-replayed, 1000 timed steps after the settle), SURVEY 8(d): 315 B/env-step."""
    N, W = args.config2_envs, 5
    res, kname = graph_steps_leg(gb, dev, rank, world, stream, N, W, args.config2_steps, args.settle)
    res["workload"] = (f"BASELINE config 2: BallEnv step + prep_state4, random actions, {N} envs/GPU, W=5, 13 static "
                       "+ 5 dynamic obstacles, TimeLimit 1000, autoreset, hipGraph replay of be_step launches")
    add_measured(res["roofline"], newest_pmc("pmc_config2.json", kname, N), res["kernel_us_mean"], N)
    return res


def config4_leg(args, gb, dev, rank, world, stream):
    """BASELINE config 4: a FIXED batch of 262 144 envs at W=10, split over the ranks (strong
    scaling; one rank per GPU): rank r steps the contiguous global ids shard(262144, r, world)
    -- 262 144 envs at N=1, 32 768 per GPU at N=8 -- with no per-step collective; after the timed
    region the ranks' episode records are all_gathered (RCCL) and combined.  Every env's
    trajectory is that of the one-rank run (Philox keyed by global env id).  1000 graph-replayed
    be_step launches per rank; value = global envs x steps / max-over-ranks wall time."""
    from gym_ballenv_amd.distributed import shard
    G, W = args.config4_envs, 10
    off, n = shard(G, rank, world)
    res, kname = graph_steps_leg(gb, dev, rank, world, stream, n, W, args.config4_steps, args.settle,
                                 env_offset=off, global_envs=G)
    res["workload"] = (f"BASELINE config 4: BallEnv step + prep_state4, random actions, {G} envs in total at W={W} "
                       f"split over {world} rank(s) ({n} envs on rank {rank}), 13 static + 5 dynamic obstacles, "
                       "TimeLimit 1000, autoreset, hipGraph replay of be_step launches; stats all_gather after the "
                       "timed region")
    res.update({"global_envs": G, "envs_per_rank": n, "ranks": world, "scaling": "strong",
                "episodes_note": "episodes finished during the timed steps (all ranks)"})
    add_measured(res["roofline"], newest_pmc(f"pmc_config4_{n}.json", kname, n), res["kernel_us_mean"], n)
    if world == 1 and args.shard_steps > 0:
        res["shards"] = config4_shards(args, gb, dev, stream, res)
    return res


def config4_shards(args, gb, dev, stream, one):
    """The 1 -> 8 GPU curve of config 4 predicted on one GPU: each per-rank shard of the 2/4/8-GPU
    split (131 072 / 65 536 / 32 768 envs) stepped exactly as that rank would -- the LAST rank's
    global ids (contiguous shard(), the highest ids), 1000 graph-replayed be_step launches after the
    settle.  Ranks share nothing per step (no collective), so a rank's step time at N GPUs is its
    shard's one-GPU time, and the node rate is projected as global envs / shard ms per step.
    `one` is the 262 144-env leg on this GPU (the N = 1 point)."""
    from gym_ballenv_amd.distributed import shard
    G, W = args.config4_envs, 10
    out = {"what": "config 4's per-rank shards on one GPU (last rank's global ids, graph-replayed be_step "
                   "launches); projected node rate = global envs / shard ms per step (no per-step collective)",
           "one_gpu": {"envs": G, "kernel": one["kernel"], "kernel_us_mean": one["kernel_us_mean"],
                       "ms_per_step": one["ms_per_step"], "value": one["value"]}}
    rows = []
    for ranks in (2, 4, 8):
        off, n = shard(G, ranks - 1, ranks)
        r, kname = graph_steps_leg(gb, dev, 0, 1, stream, n, W, args.shard_steps, args.settle, env_offset=off)
        rf = add_measured(r["roofline"], newest_pmc(f"pmc_config4_{n}.json", kname, n), r["kernel_us_mean"], n)
        proj = G / (r["ms_per_step"] * 1e-3)
        rows.append({"gpus": ranks, "envs_per_rank": n, "env_offset": off, "kernel": kname,
                     "kernel_us_mean": r["kernel_us_mean"], "ms_per_step": r["ms_per_step"],
                     "frac": rf["frac"], "moved_frac": rf["moved_frac"], "measured_frac": rf["measured_frac"],
                     "traffic_source": rf.get("traffic_source"), "moved_source": rf["moved_source"],
                     "projected_node_env_steps_per_s": proj,
                     "projected_speedup_vs_1gpu": proj / one["value"],
                     "projected_efficiency": proj / one["value"] / ranks})
    out["by_gpus"] = rows
    return out


def large_batch_leg(args, gb, dev, rank, world, stream):
    """The headline step at 2^20 envs/GPU (W=10): ~300 MB of state and outputs, past the 256-MB
    Infinity Cache, so the PMC bytes are DRAM traffic (SURVEY 8(d) caveat)."""
    N, W = args.large_envs, args.window
    res, kname = graph_steps_leg(gb, dev, rank, world, stream, N, W, args.large_steps, args.large_steps,
                                 chunk=args.large_steps)
    res["workload"] = (f"the headline step at {N} envs/GPU, W={W} (working set past the Infinity Cache), "
                       "hipGraph replay of be_step launches")
    add_measured(res["roofline"], newest_pmc("pmc_large_batch.json", kname, N), res["kernel_us_mean"], N)
    return res


def from_reset_leg(args, gb, dev, rank, world, stream):
    """The headline step timed straight from a fresh reset, no settle (round-1 bench method): the
    first ~300 steps of a fresh batch run ~7.0 -> 6.6 us (many early collisions, more resets)."""
    res, _ = graph_steps_leg(gb, dev, rank, world, stream, args.envs, args.window, args.from_reset_steps, 0)
    res["workload"] = "the headline step, timed from a fresh reset (no untimed settle)"
    return res


def blocks_leg(args, gb, dev, rank, world, stream):
    """prep_state2 block counts (be_observe_blocks) of every env of a batch
    that has stepped (obstacles spread), u8 and f32 rows, graph-replayed launches; at --envs and at
    --large-envs (DRAM-resident).  HBM-bound: agent + goal + every obstacle read (8 + 4 (Ns + Nd) B),
    the 29-byte (u8) or 116-byte (f32) row written."""
    import ctypes as C
    import torch
    res = {}
    for N, T in ((args.envs, args.blocks_launches), (args.large_envs, max(1, args.blocks_launches // 4))):
        cfg = gb.EnvConfig()
        env = gb.BatchedBallEnv(N, 10, cfg, device=dev, seed=0xB10C5, env_offset=rank * N)
        env.reset()
        for _ in range(20):
            env.step()
        lib, ctx, st = env._lib, env._ctx, C.byref(env._st)
        leg = {}
        for kind, dt, rowb in (("u8", torch.uint8, 29), ("f32", torch.float32, 116)):
            out = torch.empty(N, 29, dtype=dt, device=dev)
            u8p, f32p = (out.data_ptr(), None) if kind == "u8" else (None, out.data_ptr())
            g = torch.cuda.CUDAGraph()
            cap = torch.cuda.Stream(dev)
            with torch.cuda.graph(g, stream=cap):
                sp = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
                for _ in range(T):
                    lib.be_observe_blocks(ctx, st, C.c_void_p(u8p), C.c_void_p(f32p), sp)
            g.replay()
            el, ms = timed_graph_steps([g], T, dev, stream, world)
            B = 8 + 4 * (cfg.num_static + cfg.num_dynamic) + rowb
            ach = B * N / (ms * 1e-3) / 1e9
            leg[kind] = {"value": T * N * world / el, "unit": "env-rows/s", "kernel_us_mean": ms * 1e3,
                         "bytes_per_env": B,
                         "roofline": moved({"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                            "frac": ach / HBM_PEAK_GBS}, B, N, ms * 1e3, None,
                                           "algorithmic (exact: state read once, row written)")}
            del g
        env.status()
        env.close()
        res[f"envs_{N}"] = leg
    res["workload"] = ("be_observe_blocks (prep_state2, examples/ball_env_reinforce.py:130-172): 29 block counts "
                       "per env from the engine state, 13 static + 5 dynamic obstacles, graph-replayed launches")
    res["kernel"] = "blocks_kernel"
    return res


def newest_pmc(suffix, kernel_sub, units):
    """The NEWEST committed PMC profile profiles/rNN_<suffix> (highest round first) taken on this
    kernel at this many units per dispatch (tools/pmc_report.py / pmc_summary.py output), with
    hbm_bytes_per_dispatch / units_per_dispatch normalised across the two formats; else None.
    Older rounds' files of the same suffix are used only when no newer one matches the kernel."""
    import glob
    import re
    found = []
    for path in glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]_" + suffix)):
        m = re.match(r"r(\d\d)_", os.path.basename(path))
        found.append((int(m.group(1)), path))
    # a round-6 `..., false>` instance (no autoreset pool) is instruction for instruction the kernel
    # of the same name without the flag in earlier rounds, so those profiles stand for it
    subs = [kernel_sub]
    if kernel_sub.endswith(", false>") or kernel_sub.endswith(", false>("):
        subs.append(kernel_sub.replace(", false>", ">"))
    for rnd, path in sorted(found, reverse=True):
        d = json.load(open(path))
        u = d.get("units_per_dispatch", d.get("envs"))
        if u != units or not any(k in (d.get("kernel") or "") for k in subs):
            continue
        d.setdefault("hbm_bytes_per_dispatch", d.get("hbm_bytes_per_launch"))
        d.setdefault("hbm_bytes_per_unit", d["hbm_bytes_per_dispatch"] / units)
        d["source"] = "committed profile " + os.path.relpath(path, ROOT)
        return d
    return None


FRAC_NOTE = ("frac > 1: SURVEY 8(d)'s per-unit figure (390 B/env-step: int32 coordinates, a stored counter) is "
             "more than this layout moves (be_step_bytes, 275 B); moved_frac is the bandwidth fraction of the "
             "bytes actually moved")


def moved(rf, B_eng, units, us, pmc, label="be_step_bytes (engine)"):
    """roofline.moved_*: the bytes a launch actually moves -- the committed PMC traffic of this kernel
    at this size when one exists (2 x FETCH_SIZE + WRITE_SIZE), else the engine's own algorithmic bytes
    (be_step_bytes) -- per launch / kernel time / 8 TB/s, beside `frac` on the SURVEY figure; a `frac`
    above 1 carries frac_note."""
    b = pmc["hbm_bytes_per_dispatch"] if pmc else B_eng * units
    rf.update({"moved_bytes_per_launch": b, "moved_source": pmc["source"] if pmc else label,
               "moved_frac": b / (us * 1e-6) / 1e9 / HBM_PEAK_GBS})
    if rf.get("frac") is not None and rf["frac"] > 1.0:
        rf["frac_note"] = FRAC_NOTE
    return rf


def board_roofline(B, N, us, pmc, steps_per_launch=1):
    """HBM roofline of a createBoard kernel plus its newest committed counters: f64-VALU work, not HBM.
    us is per step; a fused launch covers steps_per_launch steps, so its counters are scaled to one step."""
    ach = B * N / (us * 1e-6) / 1e9
    r = {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": ach / HBM_PEAK_GBS,
         "traffic": None,
         "limiter": "neither roofline: f64 VALU (featureExtractor: 7 correctly rounded sqrt, 6 exp, acos, hypot "
                    "per env-step) at one wave per SIMD"}
    if pmc:
        ws = pmc["wave_cycle_split"]
        pmc = dict(pmc, hbm_bytes_per_dispatch=pmc["hbm_bytes_per_dispatch"] / steps_per_launch)   # per step
        r.update({"traffic": pmc["hbm_bytes_per_dispatch"], "traffic_per_env_step": pmc["hbm_bytes_per_unit"],
                  "valu_insts_per_wave": pmc["per_wave"]["SQ_INSTS_VALU"],
                  "wave_cycle_split": ws, "pmc_source": pmc["source"],
                  "limiter": "neither roofline, one wave per SIMD: a wave issues VALU %.0f %% and waits (memory, "
                             "dependencies) %.0f %% of its cycles; the work is f64 (featureExtractor: 7 correctly "
                             "rounded sqrt, 6 exp, acos, hypot per env-step)" % (100 * ws["SQ_ACTIVE_INST_VALU"],
                                                                                  100 * ws["SQ_WAIT_ANY"])})
    return moved(r, B, N, us, pmc, "algorithmic (above)")


def board_leg(args, gb, dev, rank, world, stream):
    """createBoard profile (ballenv_pygame.py:314-706 + featureExtractor): step + 20 features
    for every env, random actionArray moves, 6 static obstacles, autoreset, graph replay."""
    import ctypes as C
    import torch
    N, T = args.envs, args.board_steps
    b = gb.BatchedBoard(N, 6, device=dev, seed=0xB0A2D, env_offset=rank * N, autoreset=True, time_limit=1000)
    b.reset()
    acts = torch.randint(0, 4, (T, N), dtype=torch.uint8, device=dev)
    lib = b._lib
    for t in range(10):
        b.step(acts[t])
    g = torch.cuda.CUDAGraph()
    cap = torch.cuda.Stream(dev)
    with torch.cuda.graph(g, stream=cap):
        sp = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        for t in range(T):
            lib.be_board_step(b._h, C.byref(b._st), C.c_void_p(acts[t].data_ptr()), None, C.byref(b._out), sp)
    g.replay()
    el, ms = timed_graph_steps([g], T, dev, stream, world)
    b.status()
    # bytes per env-step: agent/dist/ret/len R+W 44, goal/total/episode R 28, 6 statics R 24,
    # action R 1, reward W 8, done+truncated W 2, features W 80
    B = 44 + 28 + 4 * 6 + 1 + 10 + 80
    res = {"workload": f"createBoard profile: step + featureExtractor (20 f32), {N} envs/GPU, 6 static obstacles, "
                       "random actionArray moves, autoreset, hipGraph replay",
           "value": T * N * world / el, "unit": "env-steps/s", "ms_per_step": el / T * 1e3,
           "kernel_us_mean": ms * 1e3, "bytes_per_env_step": B, "achieved_GBs": B * N / (ms * 1e-3) / 1e9}
    kname = "board_kernel<6, false, 1, true>" if b.pool_bytes() else "board_kernel<6, false, 1, false>"
    res["kernel"] = kname
    res["roofline"] = board_roofline(B, N, ms * 1e3, newest_pmc("pmc_board_step.json", kname, N))
    if b.pool_bytes():   # ballenv.hip's pool for this profile; the fills are inside the timed graph
        res["roofline"]["autoreset_pool"] = {
            "bytes": b.pool_bytes(), "fill_period_steps": int(os.environ.get("BALLENV_POOL_PERIOD", "128")),
            "what": "every env's next two episodes' Philox resets drawn ahead by board_pool_fill (every 128 steps, "
                    "inside the replayed graph); the step kernel copies a current entry instead of running the "
                    "reset waves"}
    del g
    # the same rollout fused: be_board_rollout, 100 steps per launch with the state in registers
    Kc = min(100, T)
    b.rollout(acts[:Kc])                            # warm-up; allocates the (Kc, N, ...) buffers
    f, r, dn, info = b.rollout(acts[:Kc])
    out = gb._abi.BeBoardOut(f.data_ptr(), r.data_ptr(), dn.data_ptr(), info["truncated"].data_ptr())
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if DIST_ON:
        import torch.distributed as dist
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    ev0.record(stream)
    sp = C.c_void_p(stream.cuda_stream)
    for c0 in range(0, T - T % Kc, Kc):
        lib.be_board_rollout(b._h, C.byref(b._st), C.c_void_p(acts[c0].data_ptr()), None, Kc, C.byref(out), sp)
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    if DIST_ON:
        dist.barrier()
    el = time.perf_counter() - t0
    if DIST_ON:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    Tf = T - T % Kc
    b.status()
    res["fused"] = {"what": f"be_board_rollout, {Kc} steps per launch (state in registers; per-step features, "
                            "reward, done, truncated to (K, N, ...) buffers; bit-identical to be_board_step)",
                    "value": Tf * N * world / el, "unit": "env-steps/s", "ms_per_step": el / Tf * 1e3,
                    "kernel_us_per_step": ev0.elapsed_time(ev1) * 1e3 / Tf}
    # fused bytes per env-step: action 1 + reward 8 + done/truncated 2 + features 80, the state once per launch
    Bf = 1 + 8 + 2 + 80 + (2 * 44 + 28 + 24) / Kc
    res["fused"]["bytes_per_env_step"] = Bf
    res["fused"]["roofline"] = board_roofline(Bf, N, res["fused"]["kernel_us_per_step"],
                                              newest_pmc("pmc_board_rollout.json", "board_kernel<6, true",
                                                            N * Kc), steps_per_launch=Kc)
    b.close()
    return res


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    global DIST_ON
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    DIST_ON = "WORLD_SIZE" in os.environ   # under torchrun: the collectives run even at one rank
    if args.gpus != world:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world} (launch one rank per GPU: "
                         f"torchrun --nproc-per-node {args.gpus} bench.py --gpus {args.gpus}, or bench.py --gpus N alone)")

    base = board_base = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        base = cpu_baseline(args.window, args.cpu_seconds, args.cpu_procs)
        if args.board_steps > 0 and args.board_cpu_seconds > 0:
            board_base = board_cpu_baseline(args.board_cpu_seconds, args.cpu_procs)

    import torch
    import torch.distributed as dist
    import gym_ballenv_amd as gb
    from gym_ballenv_amd import _abi

    if args.dist_backend == "gloo":           # rehearsal: ranks may share a GPU
        local_rank %= max(1, torch.cuda.device_count())
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if DIST_ON:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")

    N, W = args.envs, args.window
    cfg = gb.EnvConfig()
    env = gb.BatchedBallEnv(N, W, cfg, device=dev, seed=0xBA11, env_offset=rank * N)
    B = gb.survey_step_bytes(cfg, W)          # SURVEY §8(d) per-unit figure (390 B at the defaults)
    B_eng = gb.step_bytes(cfg, W)             # what the packed layout actually moves (275 B)
    lib = _abi.lib()
    K, WU = args.steps, args.warmup
    actions = env.sample_actions(K + WU, seed=0xBA11)            # (steps, N) u8, resident in HBM
    env.reset()
    stream = torch.cuda.current_stream(dev)

    st_ref, out_ref = C.byref(env._st), C.byref(env._out)
    step_fn, ctx = lib.be_step, env._ctx
    a0, rowb = actions.data_ptr(), N

    def launch(t, s):
        rc = step_fn(ctx, st_ref, C.c_void_p(a0 + t * rowb), None, None, out_ref, s)
        if rc:
            _abi.check(rc, ctx)

    # warm-up (eager): actions rows K .. K+WU-1
    s_ptr = C.c_void_p(stream.cuda_stream)
    for t in range(WU):
        launch(K + t, s_ptr)
    torch.cuda.synchronize(dev)
    env.status()

    graphs = []
    if args.mode == "graph":
        cap = torch.cuda.Stream(dev)
        chunk = max(1, min(args.graph_chunk, K))
        for c0 in range(0, K, chunk):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=cap):
                cs = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
                for t in range(c0, min(K, c0 + chunk)):
                    launch(t, cs)
            graphs.append(g)
        torch.cuda.synchronize(dev)
        # untimed replays of the captured graphs (the first uploads them and pays the clock ramp);
        # they step the envs, like the eager warm-up above, on actions rows 0..K-1, and are
        # repeated until --settle steps have run since reset, so the timed region starts past the
        # post-reset transient (step-kernel time falls from ~7.0 to ~6.6 us over the first
        # ~300 steps of a fresh batch: fewer early collisions -> fewer reset waves) whatever
        # --steps/--warmup are
        untimed = WU
        while True:
            for g in graphs:
                g.replay()
            untimed += K
            if untimed >= args.settle:
                break
        torch.cuda.synchronize(dev)

    if args.mode != "graph":   # untimed passes of the timed command (like the graph replays above)
        untimed = WU
        while True:
            if args.mode == "loop":
                rc = lib.be_step_n(ctx, st_ref, C.c_void_p(a0), K, out_ref, s_ptr)
                if rc:
                    _abi.check(rc, ctx)
            else:
                for t in range(K):
                    launch(t, s_ptr)
            untimed += K
            if untimed >= args.settle:
                break
        torch.cuda.synchronize(dev)

    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    env.clear_stats()             # in place: `episodes` counts the timed steps' episodes only
    if DIST_ON:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ev0.record(stream)
    t0 = time.perf_counter()
    if args.mode == "loop":
        rc = lib.be_step_n(ctx, st_ref, C.c_void_p(a0), K, out_ref, s_ptr)
        if rc:
            _abi.check(rc, ctx)
    elif args.mode == "graph":
        for g in graphs:
            g.replay()            # replays on the current stream (= stream)
    else:
        for t in range(K):
            launch(t, s_ptr)
    ev1.record(stream)
    torch.cuda.synchronize(dev)   # (measured: a spin on the end event first adds ~1.5 us, tools/sync_cost.py)
    elapsed = time.perf_counter() - t0
    own_elapsed = elapsed
    # average launch duration over the timed region (events on the launch stream)
    kern_ms = ev0.elapsed_time(ev1) / K
    if DIST_ON:
        dist.barrier()
    n_devices = 1
    per_rank_rows = None
    if DIST_ON:
        el = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
        elapsed = float(el.item())
        t_ag = time.perf_counter()
        per_rank = gb.gather_stats(env.stats_record())            # RCCL all_gather of episode returns
        torch.cuda.synchronize(dev)
        ag_us = (time.perf_counter() - t_ag) * 1e6
        ep = gb.combine_stats(per_rank)
        per_rank_rows = rank_rows(dev, {"local_rank": local_rank, "envs": N, "env_offset": rank * N,
                                        "kernel_us_mean": kern_ms * 1e3, "ms_per_step": own_elapsed / K * 1e3,
                                        "stats_all_gather_us": ag_us})
        n_devices = len({(r["host"], r["device_uuid"]) for r in per_rank_rows})   # distinct GPUs, not ranks
    else:
        ep = env.episode_stats()
    env.status()

    total_steps = K * N * world
    value = total_steps / elapsed
    achieved = B * N / (kern_ms * 1e-3) / 1e9                  # GB/s, algorithmic (§8(d)), per launch
    achieved_eng = B_eng * N / (kern_ms * 1e-3) / 1e9          # GB/s, engine bytes, per launch

    # HBM-side bytes per launch from the newest committed PMC passes (tools/pmc_bench.sh):
    # 2 x FETCH_SIZE (gfx950 reports half of wide reads) + WRITE_SIZE, same kernel / envs / W
    # (committed profile, used only when it was taken on the kernel this run launched, same envs/W)
    kname = env.kernel_name("step")
    headline_pool = pool_info(env)
    pmc = newest_pmc("pmc_step_kernel.json", f"::{kname}(", N)
    traffic, traffic_src = (pmc["hbm_bytes_per_dispatch"], pmc["source"]) if pmc else (None, None)

    cold_res = cold_actions_leg(args, env, lib, dev, stream, world, B) if args.cold_steps > 0 else None
    eager_res = eager_step_leg(args, gb, dev, rank, world, stream, kern_ms * 1e3) if args.eager_steps > 0 else None
    c2_res = config2_leg(args, gb, dev, rank, world, stream) if args.config2_steps > 0 else None
    c4_res = config4_leg(args, gb, dev, rank, world, stream) if args.config4_steps > 0 else None
    large_res = large_batch_leg(args, gb, dev, rank, world, stream) if args.large_steps > 0 else None
    fresh_res = from_reset_leg(args, gb, dev, rank, world, stream) if args.from_reset_steps > 0 else None
    pol_res = policy_leg(args, gb, dev, rank, world, stream) if args.policy_steps > 0 else None
    board_res = board_leg(args, gb, dev, rank, world, stream) if args.board_steps > 0 else None
    if board_res is not None:
        board_res["cpu_baseline"] = board_base
    roll_res = rollout_leg(args, gb, dev, rank, world, stream) if args.rollout_steps > 0 else None
    if roll_res is not None and world == 1:
        # the same fused mode at the other BASELINE sizes (SURVEY 8(d) reports it separately): config 2
        # (4 096 envs, W=5: rolloutw_kernel) and config 4's 8-GPU shard (32 768 envs at the last rank's ids)
        from gym_ballenv_amd.distributed import shard
        roll_res["config2"] = rollout_leg(args, gb, dev, 0, 1, stream, N=args.config2_envs, W=5, env_offset=0,
                                          pmc_suffix="pmc_rollout_config2.json",
                                          label=f"BASELINE config 2: random-action rollout, {args.config2_envs} envs, W=5")
        off8, n8 = shard(262144, 7, 8)       # BASELINE config 4's batch, whatever --config4-envs says
        roll_res["shard_32768"] = rollout_leg(args, gb, dev, 0, 1, stream, N=n8, W=10, env_offset=off8,
                                              pmc_suffix=f"pmc_rollout_shard_{n8}.json",
                                              label=f"config 4's 8-GPU shard: random-action rollout, {n8} envs "
                                                    f"(global ids {off8}..{off8 + n8 - 1}), W=10")
        if base is not None:   # the host port at the same windows (cpu_baseline.by_window)
            for key, w in (("config2", 5), ("shard_32768", 10)):
                bw = base["by_window"].get(f"W={w}")
                if bw:
                    roll_res[key]["cpu_baseline_ref"] = {"window": w, "aggregate": bw["aggregate"],
                                                         "per_core": bw["per_core_mean"], "cores": base["cores"],
                                                         "source": f"cpu_baseline.by_window.W={w}"}
    blocks_res = blocks_leg(args, gb, dev, rank, world, stream) if args.blocks_launches > 0 else None

    if rank == 0:
        line = {
            "metric": "env-steps/sec (whole node), batch=65536 envs, window=10; achieved HBM GB/s",
            "value": value, "unit": "env-steps/s", "n_gpus": n_devices, "ranks": world, "steps": K, "warmup": WU,
            "untimed_steps": untimed,
            "ms_per_step": elapsed / K * 1e3, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "int16x2+f64", "data": "synthetic",
            "config": {"workload": f"BallEnv step + prep_state4 window, random actions, {N} envs/GPU, W={W}, "
                                   "13 static + 5 dynamic obstacles, TimeLimit 1000, autoreset",
                       "envs_per_gpu": N, "global_envs": N * world, "window": W,
                       "parallelism": f"env-shard x{world} (no per-step collective)",
                       "launch": {"loop": "be_step_n: K be_step launches queued by the library's C loop",
                                  "graph": "hipGraph replay of be_step launches",
                                  "eager": "one ctypes be_step call per step"}[args.mode]},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "bytes_per_env_step": B, "bytes_source": "SURVEY.md 8(d): 82+8*Ns+20*Nd+4+W^2",
                         "engine_bytes_per_env_step": B_eng, "engine_achieved": achieved_eng,
                         "engine_frac": achieved_eng / HBM_PEAK_GBS, "kernel_us_mean": kern_ms * 1e3,
                         "kernel": kname, "traffic_source": traffic_src,
                         "measured_frac": (traffic / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBS) if traffic else None,
                         "measured_note": "measured_frac = PMC bytes per launch (2 x FETCH_SIZE + WRITE_SIZE) / kernel "
                                          "time / 8 TB/s; at 65 536 envs those bytes are Infinity-Cache (MALL) "
                                          "fabric requests, not DRAM: see large_batch for a DRAM-resident point"},
            "cpu_baseline": base,
            "episodes": ep,
            "cold_action_rows": cold_res,
            "eager_step": eager_res,
            "config2": c2_res,
            "config4": c4_res,
            "large_batch": large_res,
            "from_reset": fresh_res,
            "policy_rollout": pol_res,
            "board_profile": board_res,
            "fused_rollout": roll_res,
            "blocks_obs": blocks_res,
        }
        moved(line["roofline"], B_eng, N, kern_ms * 1e3, pmc)
        if headline_pool:
            line["roofline"]["autoreset_pool"] = headline_pool
        line["episodes_note"] = "episodes finished during the timed steps (all ranks)"
        if per_rank_rows is not None:
            # N > 1: each rank's own timing (the line's ms_per_step is the max of these), its GPU, and
            # the stats all_gather's wall time -- a scaling run explains its own curve
            line["per_rank"] = per_rank_rows
            line["dist_backend"] = args.dist_backend
            line["rccl_world_size"] = dist.get_world_size() if args.dist_backend == "nccl" else None
        print(json.dumps(line), flush=True)
    env.close()
    if DIST_ON:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
