"""HBM-side bytes per unit of one kernel from rocprofv3 --pmc passes (one pass per counter).

    python tools/pmc_kernel.py <pass root> <kernel-name regex> <units per dispatch> [out.json]
<pass root>/FETCH_SIZE/**/counter_collection.csv and <pass root>/WRITE_SIZE/**/... ;
traffic = 2 * FETCH_SIZE + WRITE_SIZE (kB; gfx950 FETCH_SIZE reports half of wide reads,
MI355X_MICROARCH.md), averaged over the kernel's dispatches, divided by units per dispatch.
"""
import csv
import glob
import json
import os
import re
import statistics
import sys

root, pat, units = sys.argv[1], sys.argv[2], float(sys.argv[3])
vals, name = {}, None
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    f = glob.glob(os.path.join(root, c, "**", "*counter_collection.csv"), recursive=True)[0]
    per = {}
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] == c and re.search(pat, r["Kernel_Name"]):
            name = r["Kernel_Name"]
            per[int(r["Dispatch_Id"])] = per.get(int(r["Dispatch_Id"]), 0.0) + float(r["Counter_Value"])
    vals[c] = statistics.mean(per.values()) * 1024.0
    vals[c + "_n"] = len(per)
hbm = 2 * vals["FETCH_SIZE"] + vals["WRITE_SIZE"]
out = {"kernel": name, "dispatches": vals["FETCH_SIZE_n"], "units_per_dispatch": units,
       "fetch_size_bytes_reported": vals["FETCH_SIZE"], "write_size_bytes": vals["WRITE_SIZE"],
       "hbm_bytes_per_dispatch": hbm, "hbm_bytes_per_unit": hbm / units,
       "note": "2 x FETCH_SIZE + WRITE_SIZE (gfx950 FETCH_SIZE = half of wide reads)"}
print(json.dumps(out))
if len(sys.argv) > 4:
    json.dump(out, open(sys.argv[4], "w"), indent=1)
