"""Per-kernel summary of tools/pmc_passes.sh passes.

    python tools/pmc_report.py <pass root> <kernel regex> <units per dispatch> [--first N] [--grid G] [--out f.json]

Averages each counter over the first N matching dispatches (default: all), per dispatch; --grid keeps
only dispatches of that Grid_Size (threads), so another leg's launches of the same kernel at another
batch size (the bench's short headline leg beside a config-4 shard leg) stay out of the average.
HBM bytes = 2 x FETCH_SIZE + WRITE_SIZE (kB; gfx950 FETCH_SIZE reports half of wide reads,
MI355X_MICROARCH.md 'HBM').  SQ_*_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles,
SQ_VALU_MFMA_BUSY_CYCLES cycles (MI355X_MICROARCH.md 'per-instruction cycle constants');
effective clock = GRBM_GUI_ACTIVE / 8 XCDs / kernel time (reads high below ~0.3 ms dispatches).
"""
import argparse
import csv
import glob
import json
import os
import re
import statistics

ap = argparse.ArgumentParser()
ap.add_argument("root")
ap.add_argument("pattern")
ap.add_argument("units", type=float)
ap.add_argument("--first", type=int, default=0)
ap.add_argument("--grid", type=int, default=0)
ap.add_argument("--out")
a = ap.parse_args()

vals, name, ndisp = {}, None, {}
for d in sorted(glob.glob(os.path.join(a.root, "*", ""))):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        continue
    per = {}
    for r in csv.DictReader(open(files[0])):
        if re.search(a.pattern, r["Kernel_Name"]) and (not a.grid or int(r["Grid_Size"]) == a.grid):
            name = r["Kernel_Name"]
            key = (r["Counter_Name"], int(r["Dispatch_Id"]))
            per[key] = per.get(key, 0.0) + float(r["Counter_Value"])
    ctrs = sorted({c for c, _ in per})
    for c in ctrs:
        ids = sorted(i for cc, i in per if cc == c)
        if a.first:
            ids = ids[:a.first]
        vals[c] = statistics.mean(per[(c, i)] for i in ids)
        ndisp[c] = len(ids)

out = {"kernel": name, "units_per_dispatch": a.units, "grid_size": a.grid or None, "dispatches": ndisp,
       "counters_per_dispatch": vals}
g = vals.get
if "FETCH_SIZE" in vals and "WRITE_SIZE" in vals:
    hbm = (2 * vals["FETCH_SIZE"] + vals["WRITE_SIZE"]) * 1024.0
    out.update({"hbm_bytes_per_dispatch": hbm, "hbm_bytes_per_unit": hbm / a.units})
if g("SQ_WAVES"):
    w = vals["SQ_WAVES"]
    out["per_wave"] = {k: vals[k] / w for k in ("SQ_INSTS_VALU", "SQ_INSTS_MFMA", "SQ_INSTS_LDS", "SQ_INSTS_SALU")
                       if k in vals}
if g("SQ_WAVE_CYCLES"):
    wc = vals["SQ_WAVE_CYCLES"]
    out["wave_cycle_split"] = {k: vals[k] / wc for k in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
                                                         "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS",
                                                         "SQ_WAIT_INST_LDS") if k in vals}
if g("GRBM_GUI_ACTIVE"):
    kc = vals["GRBM_GUI_ACTIVE"] / 8.0                   # GPU cycles per dispatch (summed over 8 XCDs)
    out["gpu_cycles_per_dispatch"] = kc
    if "SQ_VALU_MFMA_BUSY_CYCLES" in vals:               # summed over the 1024 SIMDs (cycles)
        out["mfma_busy_frac_est"] = vals["SQ_VALU_MFMA_BUSY_CYCLES"] / (kc * 1024.0)
    if "SQ_ACTIVE_INST_VALU" in vals:                    # quad-cycles, summed over waves
        out["valu_active_per_simd_frac_est"] = 4.0 * vals["SQ_ACTIVE_INST_VALU"] / (kc * 1024.0)
if g("SQ_LDS_IDX_ACTIVE"):
    out["lds_bank_conflict_frac"] = vals.get("SQ_LDS_BANK_CONFLICT", 0.0) / vals["SQ_LDS_IDX_ACTIVE"]
print(json.dumps(out, indent=1))
if a.out:
    json.dump(out, open(a.out, "w"), indent=1)
