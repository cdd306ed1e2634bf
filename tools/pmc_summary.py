#!/usr/bin/env python3
"""Per-kernel median of every counter in rocprofv3 --pmc output directories.

    python tools/pmc_summary.py DIR [DIR ...] [--kernel SUBSTR]

Counter values of one dispatch are summed over their instances (XCDs, SEs);
the median is over dispatches of the same kernel."""
import csv
import collections
import glob
import os
import statistics
import sys


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    ksub = None
    if "--kernel" in sys.argv:
        ksub = sys.argv[sys.argv.index("--kernel") + 1]
        args.remove(ksub)
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    names = {}
    for d in args:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                k = r.get("Kernel_Name", "")
                if ksub and ksub not in k:
                    continue
                did = r.get("Dispatch_Id", r.get("Correlation_Id"))
                per[(k, did)][r["Counter_Name"]] += float(r["Counter_Value"])
                names[k] = k
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for (k, _), cs in per.items():
        for c, v in cs.items():
            agg[k][c].append(v)
    for k in sorted(agg):
        short = k.split("(")[0][:90]
        n = max(len(v) for v in agg[k].values())
        print(f"{short}  [{n} dispatches]")
        for c in sorted(agg[k]):
            print(f"    {c:28s} {statistics.median(agg[k][c]):16.4g}")


if __name__ == "__main__":
    main()
