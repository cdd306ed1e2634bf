#!/usr/bin/env python3
"""Table of per-kernel PMC counters over the measured batches of
tools/gpu_pmc_mix.sh runs: for each kernel named in PMC_KERN and each counter,
the mean over the last 3 batches of every mix:seed run."""
import collections
import csv
import glob
import os
import sys

out = sys.argv[1]
runs = [r.replace(":", "_") for r in os.environ["PMC_RUNS"].split()]
kern = os.environ["PMC_KERN"].split(",")
data = {}
for r in runs:
    rows = []
    for f in glob.glob(os.path.join(out, r, "**", "*counter_collection.csv"), recursive=True):
        rows += [x for x in csv.DictReader(open(f)) if "gvs::" in x["Kernel_Name"]]
    key = "Dispatch_Id" if rows and "Dispatch_Id" in rows[0] else "Correlation_Id"
    per = collections.defaultdict(dict)
    names = {}
    for x in rows:
        d = int(x[key])
        names[d] = x["Kernel_Name"].split("(")[0].replace("void ", "").replace("gvs::", "")
        per[d][x["Counter_Name"]] = per[d].get(x["Counter_Name"], 0.0) + float(x["Counter_Value"])
    byk = collections.defaultdict(list)
    for d in sorted(per):
        byk[names[d]].append(per[d])
    data[r] = byk
ctrs = sorted({c for byk in data.values() for L in byk.values() for v in L for c in v})
allk = sorted({k for byk in data.values() for k in byk if any(k.startswith(p) for p in kern)})
for k in allk:
    print(k)
    for c in ctrs:
        cells = []
        for r in runs:
            L = data[r].get(k, [])
            vals = [v.get(c, 0.0) for v in L]
            nb = sum(1 for _ in data[r].get("k_copy", [])) or 1
            per_b = max(1, len(vals) // nb)
            meas = vals[-3 * per_b:]
            cells.append(f"{r}={sum(meas) / max(1, len(meas)):.1f}")
        print(f"  {c:24s} " + "  ".join(cells))
