"""Step-kernel time per (envs, W, lanes-per-env override) in ONE process: bench.py's graph-replay
method (graph_steps_leg), the override env var set before each context is created.

    python tools/lane_sweep.py --window 5 --envs 4096,8192 --lanes 1,4,8 [--steps 1000] [--var BALLENV_STEP5_LPE]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

ap = argparse.ArgumentParser()
ap.add_argument("--window", type=int, default=5)
ap.add_argument("--envs", default="4096")
ap.add_argument("--lanes", default="1,8")
ap.add_argument("--steps", type=int, default=1000)
ap.add_argument("--settle", type=int, default=400)
ap.add_argument("--var", default="")
ap.add_argument("--reps", type=int, default=2)
ap.add_argument("--rollout", action="store_true", help="time be_rollout (bench.py's fused leg) instead of be_step")
a = ap.parse_args()
var = a.var or (("BALLENV_ROLLOUT5_LPE" if a.rollout else "BALLENV_STEP5_LPE") if a.window == 5 else "BALLENV_STEP_LPE")

import torch  # noqa: E402
import bench  # noqa: E402
import gym_ballenv_amd as gb  # noqa: E402

dev = torch.device("cuda", 0)
stream = torch.cuda.current_stream(dev)
for rep in range(a.reps):
    for n in [int(x) for x in a.envs.split(",")]:
        for l in a.lanes.split(","):
            os.environ[var] = l
            if a.rollout:
                args = argparse.Namespace(envs=n, window=a.window, rollout_steps=a.steps, rollout_chunk=100)
                r = bench.rollout_leg(args, gb, dev, 0, 1, stream)
                k = r["kernel"]
                r["kernel_us_mean"] = r["kernel_us_per_step"]
                r["roofline"] = {"frac": r["frac"]}
            else:
                r, k = bench.graph_steps_leg(gb, dev, 0, 1, stream, n, a.window, a.steps, a.settle)
            print(json.dumps({"rep": rep, "envs": n, "window": a.window, var: l, "kernel": k,
                              "kernel_us": round(r["kernel_us_mean"], 3), "value": r["value"],
                              "frac390": r["roofline"]["frac"]}), flush=True)
