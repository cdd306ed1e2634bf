#!/bin/bash
# tools/bubble_probe.hip: TCC_BUBBLE and read requests by where a pass reads its slot lines
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/bubble
rm -rf "$O"; mkdir -p "$O"
timeout -s KILL 120 rocprofv3 --pmc TCC_BUBBLE_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum \
  -d "$O/a" -o run --output-format csv -- ./tools/bubble_probe > "$O/a.log" 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum \
  -d "$O/b" -o run --output-format csv -- ./tools/bubble_probe > "$O/b.log" 2>&1 || exit 1
python3 - <<'PY' | tee "$O/summary.txt"
import csv, glob, collections
for d in ("a", "b"):
    rows = []
    for f in glob.glob(f"gpurun_out/bubble/{d}/**/*counter_collection.csv", recursive=True):
        rows += list(csv.DictReader(open(f)))
    per = collections.defaultdict(dict); kn = {}
    for r in rows:
        i = int(r["Dispatch_Id"]); kn[i] = r["Kernel_Name"].split("(")[0].replace("void ", "")
        per[i][r["Counter_Name"]] = per[i].get(r["Counter_Name"], 0) + float(r["Counter_Value"])
    by = collections.defaultdict(list)
    for i in sorted(per):
        if "k_pass" in kn[i]: by[kn[i]].append(per[i])
    for k, L in sorted(by.items()):
        print(d, k, " ".join(f"{c}={[int(x[c]) for x in L]}" for c in L[0]))
PY
