#!/bin/bash
# FETCH_SIZE of whole-row gathers in different orders (tools/fetch_probe.hip)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/fetch_probe
mkdir -p "$O"
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE -d "$O/f" -o run --output-format csv -- ./tools/fetch_probe > "$O/f.log" 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_HIT_sum TCC_MISS_sum -d "$O/r" -o run --output-format csv -- ./tools/fetch_probe > "$O/r.log" 2>&1 || exit 1
python3 - <<'PY'
import csv, glob, collections
for d in ["f", "r"]:
    rows = []
    for f in glob.glob(f"gpurun_out/fetch_probe/{d}/**/*counter_collection.csv", recursive=True):
        rows += list(csv.DictReader(open(f)))
    per = collections.defaultdict(dict)
    for r in rows:
        if "k_rows" not in r["Kernel_Name"]:
            continue
        per[(int(r.get("Dispatch_Id", 0)), r["Kernel_Name"][:9])][r["Counter_Name"]] = float(r["Counter_Value"])
    for i, k in enumerate(sorted(per)):
        print(d, k[1], ["seq", "perm", "scatter", "mixed"][(i // 2) % 4], per[k])
PY
