#!/usr/bin/env python3
"""Diagnostic: run tools/oblivious_probe.py for every request mix under
`rocprofv3 --pmc <counters>` and print, per kernel and counter, the range over
the measured batches of each mix.  Used to attribute a byte-counter difference
(e.g. instruction fetch vs vector data vs scalar data).

    python tools/counter_mix.py OUTDIR COUNTER [COUNTER ...]
"""
import csv
import collections
import glob
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROBE = os.path.join(ROOT, "tools", "oblivious_probe.py")
MIXES = ["main", "all_create", "all_miss_read", "hot_next", "deletes"]


def run(outdir, counters, mix):
    d = os.path.join(outdir, mix)
    cmd = ["rocprofv3", "--pmc"] + counters + ["-d", d, "-o", "run", "--output-format", "csv",
                                                 "--", sys.executable, PROBE, mix]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT)
    if r.returncode != 0:
        sys.exit(r.stdout[-3000:] + r.stderr[-3000:])
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        rows += [r for r in csv.DictReader(open(f)) if "gvs::" in r.get("Kernel_Name", "")]
    key = "Dispatch_Id" if "Dispatch_Id" in rows[0] else "Correlation_Id"
    per = collections.defaultdict(dict)
    order = []
    for r in rows:
        did = int(r[key])
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("gvs::", "")
        if did not in per:
            order.append((did, name))
        per[did][r["Counter_Name"]] = per[did].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    order.sort()
    return [(name, per[did]) for did, name in order]


def main():
    outdir, counters = sys.argv[1], sys.argv[2:]
    res = {m: run(outdir, counters, m) for m in MIXES}
    ref = res["main"]
    nb = sum(1 for k, _ in ref if k == "k_copy")
    per_batch = len(ref) // nb
    print(f"batches per run: {nb}, kernels per batch: {per_batch}")
    for c in counters:
        print(f"== {c}  (last 3 batches per mix; prefill batch 4 in brackets)")
        for idx in range(per_batch):
            k = ref[idx][0]
            cells = []
            for m in MIXES:
                vals = [res[m][b * per_batch + idx][1].get(c, float("nan")) for b in range(nb)]
                cells.append(f"{m}=[{vals[nb - 4]:.0f}] {min(vals[-3:]):.0f}..{max(vals[-3:]):.0f}")
            print(f"  {k[:30]:30s} " + "  ".join(cells))


if __name__ == "__main__":
    main()
