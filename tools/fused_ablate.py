"""Time the fused config-5 rollout (be_policy_rollout, 65536 envs, W=10, reference
Policy(10)) under ablation bits -- a diagnostics build reads them (BE_DIAG_SKIP):

    python tools/fused_ablate.py --build            # tools/diag/skip/libballenv.so
    BALLENV_LIB=tools/diag/skip/libballenv.so python tools/fused_ablate.py [dbg ...]
dbg bits (csrc/ballenv.hip): 2048 every env on the empty-window table (no MFMA tiles),
4096 no select_action tail (a fixed action hash), 8192 no block barriers (with 2048 only),
0x20000 tile_forward without MFMA, 0x40000 tile_forward without head FMAs.
``--build [name:flag ...]`` also builds tools/diag/skip_<name>/ with extra compile flags.
Also times the tape-driven be_rollout of the same envs for reference.  Outputs under
ablation are wrong by design; only the time is meaningful.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def build(unrolls):
    from gym_ballenv_amd.build import build_library
    for u in [None, *unrolls]:
        sub, flags = ("skip", ["-DBE_DIAG_SKIP"]) if u is None else (f"skip_{u.split(':')[0]}", ["-DBE_DIAG_SKIP", u.split(':', 1)[1]])
        out = os.path.join(ROOT, "tools", "diag", sub, "libballenv.so")
        os.makedirs(os.path.dirname(out), exist_ok=True)
        build_library(extra_flags=flags, out=out)


def main():
    import torch
    import gym_ballenv_amd as gb
    from gym_ballenv_amd.policy import Policy, reference_weights
    dbgs = [int(x, 0) for x in sys.argv[1:]] or [0]
    N, W, T = int(os.environ.get("ENVS", 65536)), 10, 200
    dev = torch.device("cuda:0")
    pol = Policy.from_npz(reference_weights(W), W)
    if os.environ.get("RANDOM_POLICY"):
        torch.manual_seed(0)
        pol = Policy(W)
    if os.environ.get("ANALYZE"):   # lit-window envs per 256-env block and step (the MFMA tiles' load)
        env = gb.BatchedBallEnv(N, W, gb.EnvConfig(), device=dev, seed=0xBA11)
        env.reset()
        ro = gb.Rollout(env, pol, horizon=T, backend="fused", chunk=100, record_obs=True)
        ro.run()
        ro.run()
        lit = (ro.obs[:T, :, 4:].amax(-1) > 0).reshape(T, N // 256, 256).sum(-1).float()   # (T, blocks)
        tiles = torch.ceil(lit / 16)
        print(f"lit envs per block-step: mean {lit.mean():.1f} p50 {lit.median():.0f} p99 "
              f"{lit.flatten().kthvalue(int(0.99 * lit.numel())).values:.0f} max {lit.max():.0f}; "
              f"tiles per block-step mean {tiles.mean():.2f}, per step max over blocks mean "
              f"{tiles.amax(1).mean():.2f}; sum over steps per block: mean {tiles.sum(0).mean():.0f} "
              f"max {tiles.sum(0).max():.0f}", flush=True)
        ro.close()
        env.close()
    for dbg in dbgs:
        os.environ["BALLENV_DEBUG_SKIP"] = str(dbg)
        env = gb.BatchedBallEnv(N, W, gb.EnvConfig(), device=dev, seed=0xBA11)
        os.environ.pop("BALLENV_DEBUG_SKIP")
        env.reset()
        ro = gb.Rollout(env, pol, horizon=T, backend="fused", chunk=100)
        ro.run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        ro.run()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / T * 1e3
        dense = float((ro.obs[:, :, 4:].amax(-1) > 0).float().mean()) if ro.obs is not None else float("nan")
        n_done = int(ro.dones.sum())
        acts = ro.actions.clone()
        ro.close()
        obs, rew, done, _ = env.rollout(acts[:100])
        env.rollout(acts[100:])
        torch.cuda.synchronize()
        e0.record()
        env.rollout(acts[:100])
        env.rollout(acts[100:])
        e1.record()
        torch.cuda.synchronize()
        us_tape = e0.elapsed_time(e1) / T * 1e3
        print(f"dbg={dbg}: fused policy rollout {us:.2f} us/step (dones {n_done}/{T * N}); "
              f"be_rollout on the same actions {us_tape:.2f} us/step", flush=True)
        env.close()


if __name__ == "__main__":
    if "--build" in sys.argv:
        build(sys.argv[2:])
    else:
        main()
