"""Per-region kernel averages from a rocprofv3 kernel trace (run_kernel_trace.csv) of the default
`python3 bench.py` command: the headline's timed region, config 2's, config 4's and the 2^20-env leg's.

    python tools/trace_regions.py <kernel_trace.csv> [--warmup 100] [--untimed 1000] [--steps 1000]

bench.py's headline leg launches the step kernel `warmup` times eagerly, replays the captured graph
for `untimed` steps (settle), then times `steps` launches: launches warmup+untimed+1 ..
warmup+untimed+steps of the headline kernel are the timed region.  The config-2 leg is the last 1000
launches of its kernel; config 4 at one rank (262 144 envs, the one-lane kernel without the pool), its
per-rank shards (131 072 envs one-lane with the pool, 32 768 envs step2_kernel) and the 2^20-env leg
are the last 1000 (200) launches of that kernel at that grid size (threads: Grid_Size; the one-lane
kernel runs 1 thread per env, step2_kernel 2)."""
import argparse
import csv
import statistics
from collections import defaultdict

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--warmup", type=int, default=100)
ap.add_argument("--untimed", type=int, default=1000)
ap.add_argument("--steps", type=int, default=1000)
a = ap.parse_args()

runs = defaultdict(list)
by_grid = defaultdict(list)
for r in csv.DictReader(open(a.trace)):
    t = (int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
    runs[r["Kernel_Name"]].append(t)
    g = r.get("Grid_Size", r.get("Grid_Size_X"))   # (counter CSVs: Grid_Size; kernel traces: Grid_Size_X)
    if g:
        by_grid[(r["Kernel_Name"], int(g))].append(t)
for k in list(runs) + list(by_grid):
    (runs if k in runs else by_grid)[k].sort()


def avg_us(launches):
    return statistics.mean((e - s) for s, e in launches) / 1e3


def find(prefix):
    return next((k for k in runs if prefix in k), None)


def fills_in(t0, t1, grid, name="pool_fill_kernel"):
    """the autoreset pool's fill launches (pool_fill_kernel / board_pool_fill, one lane per env) inside [t0, t1]"""
    out = []
    for k in runs:
        if name in k:
            out += [x for x in by_grid.get((k, grid), []) if t0 <= x[0] and x[1] <= t1]
    return out


head = find("step2_kernel<10, 13, 5, true>") or find("step2_kernel<10, 13, 5")
if head:
    L = runs[head]
    lo = a.warmup + a.untimed
    reg = L[lo:lo + a.steps]
    print(f"{head}: {len(L)} launches in the whole command; the headline's timed region (launches "
          f"{lo + 1}..{lo + len(reg)}) averages {avg_us(reg):.3f} us per launch; "
          f"65536 x 390 B / that = {65536 * 390 / (avg_us(reg) * 1e-6) / 1e12:.2f} TB/s")
    fl = fills_in(reg[0][0], reg[-1][1], 65536)
    if fl:
        per = (sum(e - s for s, e in reg) + sum(e - s for s, e in fl)) / len(reg) / 1e3
        print(f"  + {len(fl)} pool_fill_kernel launches in that region, {avg_us(fl):.3f} us each: "
              f"{per:.3f} us of kernel time per step, the fills included")
for prefix, n, grid, last, what in (("be_kernel<10, 0, 13, 5, false>", 262144, 262144, 1000, "config 4 at one rank"),
                                    ("be_kernel<10, 0, 13, 5, true>", 131072, 131072, 1000, "config 4's 2-GPU shard"),
                                    ("step2_kernel<10, 13, 5, true>", 32768, 65536, 1000, "config 4's 8-GPU shard"),
                                    ("be_kernel<10, 0, 13, 5, false>", 1 << 20, 1 << 20, 200, "2^20 envs, large_batch")):
    k = find(prefix)
    L = by_grid.get((k, grid), [])
    if len(L) >= last:
        reg = L[-last:]
        print(f"{k} ({what}, {n} envs): the last {last} launches at that size average {avg_us(reg):.3f} us; "
              f"{n} x 390 B / that = {n * 390 / (avg_us(reg) * 1e-6) / 1e12:.2f} TB/s")
for prefix, last, what in (("stepw_kernel<5, 13, 5, 8, true>", 1000, "config 2, 4096 envs, W=5"),
                           ("board_kernel<6, false, 1, true>", 1000, "createBoard step, 65536 envs"),
                           ("board_kernel<6, true, 1", 10, "createBoard fused, 100 steps per launch"),
                           ("rollout_kernel<10, 13, 5, 13, 2, 10>", 10, "config 5 fused, 100 steps per launch"),
                           ("blocks_kernel", 200, "prep_state2 blocks (last leg size)")):
    k = find(prefix)
    if k:
        L = runs[k]
        print(f"{k} ({what}): {len(L)} launches; the last {min(last, len(L))} average {avg_us(L[-last:]):.3f} us")
        if prefix.startswith("board_kernel<6, false"):
            reg = L[-last:]
            fl = fills_in(reg[0][0], reg[-1][1], 65536, "board_pool_fill")
            if fl:
                per = (sum(e - s for s, e in reg) + sum(e - s for s, e in fl)) / len(reg) / 1e3
                print(f"  + {len(fl)} board_pool_fill launches among them, {avg_us(fl):.3f} us each: "
                      f"{per:.3f} us of kernel time per step, the fills included")
