"""Per-launch HBM-side bytes of the step kernel from tools/pmc_bench.sh's passes.

traffic = 2 * FETCH_SIZE + WRITE_SIZE  (kB -> bytes; on gfx950 FETCH_SIZE reports half the
bytes of wide coalesced reads: MI355X_MICROARCH.md "HBM"), averaged over the step-kernel
dispatches of the bench's timed region (warm-up and reset dispatches skipped)."""
import csv
import re
import glob
import json
import os
import statistics
import sys

root = sys.argv[1]
argv = sys.argv[2:]
envs = int(argv[argv.index("--envs") + 1]) if "--envs" in argv else 65536
window = int(argv[argv.index("--window") + 1]) if "--window" in argv else 10
steps = int(argv[argv.index("--steps") + 1])
vals = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    f = glob.glob(os.path.join(root, c, "**", "*counter_collection.csv"), recursive=True)[0]
    rows = [r for r in csv.DictReader(open(f)) if re.search(rf"(be_kernel<{window}, 0[,>]|step2_kernel<{window}, )", r["Kernel_Name"])
            and r["Counter_Name"] == c]
    kname = rows[0]["Kernel_Name"] if rows else None
    per = {}
    for r in rows:   # one row per dispatch (summed over instances if split)
        per[int(r["Dispatch_Id"])] = per.get(int(r["Dispatch_Id"]), 0.0) + float(r["Counter_Value"])
    ids = sorted(per)[-steps:]                  # the timed region's launches
    vals[c] = statistics.mean(per[i] for i in ids) * 1024.0
    vals[c + "_dispatches"] = len(ids)
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gym_ballenv_amd.config import EnvConfig, step_bytes   # noqa: E402
algo = step_bytes(EnvConfig(), window) * envs
out = {"kernel": kname, "envs": envs, "window": window,
       "fetch_size_bytes_reported": vals["FETCH_SIZE"], "write_size_bytes": vals["WRITE_SIZE"],
       "hbm_bytes_per_launch": 2 * vals["FETCH_SIZE"] + vals["WRITE_SIZE"],
       "algorithmic_bytes_per_launch": algo, "dispatches": vals["FETCH_SIZE_dispatches"],
       "note": "2 x FETCH_SIZE + WRITE_SIZE (gfx950 FETCH_SIZE = half of wide reads); Infinity-Cache hits "
               "are counted as fabric traffic"}
out["traffic_over_algorithmic"] = out["hbm_bytes_per_launch"] / algo
json.dump(out, open(os.path.join(root, "pmc_step_kernel.json"), "w"), indent=1)
print(json.dumps(out))
