#!/usr/bin/env python3
"""Per-kernel request counters of tools/gpu_req_diag.sh runs: for every kernel
launch position of the last batch, each counter's value per run; a line is
flagged when the spread across mixes exceeds the spread between the two main
runs (same mix, different seeds)."""
import collections
import csv
import glob
import os
import sys

out = sys.argv[1]
runs = [r.replace(":", "_") for r in os.environ["REQ_RUNS"].split()]
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
    seq = [(names[d], per[d]) for d in sorted(per)]
    # last batch: from the last k_copy on
    last = max(i for i, (n, _) in enumerate(seq) if n == "k_copy")
    data[r] = seq[last:]
ref = data[runs[0]]
ctrs = sorted({c for _, v in ref for c in v})
for i, (k, _) in enumerate(ref):
    for c in ctrs:
        vals = [data[r][i][1].get(c, 0.0) if i < len(data[r]) else float("nan") for r in runs]
        same = abs(vals[0] - vals[1])
        spread = max(vals) - min(vals)
        flag = "  <-- MIX" if spread > same + 0.5 else ""
        print(f"{i:3d} {k[:34]:34s} {c:24s} " + " ".join(f"{v:12.0f}" for v in vals) + flag)
