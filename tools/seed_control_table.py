# Table of the seed-vs-mix FETCH_SIZE control (DESIGN.md §3 "Results"): reads
# gpurun_out/r02c/<mix>_<seed>/ from rocprofv3 --pmc FETCH_SIZE runs of
# tools/oblivious_probe.py <mix> --seed <seed> --log2n 20 --batch 32768 --shards 2.
import csv, glob, os, sys
base = "gpurun_out/r02c"
runs = ["main_1234", "main_99", "main_5", "all_miss_read_1234", "all_miss_read_99", "all_miss_read_5"]
data = {}
for r in runs:
    files = glob.glob(os.path.join(base, r, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        continue
    rows = []
    for f in files:
        rows += list(csv.DictReader(open(f)))
    rows = [x for x in rows if "gvs::" in x["Kernel_Name"]]
    key = "Dispatch_Id" if "Dispatch_Id" in rows[0] else "Correlation_Id"
    rows.sort(key=lambda x: int(x[key]))
    per = {}
    for x in rows:
        n = x["Kernel_Name"].split("(")[0].replace("void ", "").replace("gvs::", "")
        per.setdefault(n, []).append(float(x["Counter_Value"]))
    data[r] = per
for k in ("k_m1r_c", "k_m2x<false>", "k_m1x<false>"):
    print(k)
    for r, per in data.items():
        v = per.get(k, [])
        L = len(v) // 7
        meas = v[-3 * L:]
        print(f"  {r:20s}", [round(x, 1) for x in meas])
rk = [k for k in data.get("main_1234", {}) if k.startswith("k_rpass2")]
for k in rk:
    print(k)
    for r, per in data.items():
        v = per.get(k, [])
        L = len(v) // 7
        print(f"  {r:20s}", [round(x, 1) for x in v[-3 * L:]])
