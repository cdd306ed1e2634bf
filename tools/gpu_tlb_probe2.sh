#!/bin/bash
# tools/tlb_probe2.hip: page-table walks (uncached reads) of a random gather by span
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/tlb2
rm -rf "$O"; mkdir -p "$O"
timeout -s KILL 180 rocprofv3 --pmc TCC_UC_REQ_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_sum \
  -d "$O/a" -o run --output-format csv -- ./tools/tlb_probe2 > "$O/a.log" 2>&1 || exit 1
python3 - <<'PY' | tee "$O/summary.txt"
import csv, glob, collections
rows = []
for f in glob.glob("gpurun_out/tlb2/a/**/*counter_collection.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
per = collections.defaultdict(dict); kn = {}
for r in rows:
    i = int(r["Dispatch_Id"]); kn[i] = r["Kernel_Name"]
    per[i][r["Counter_Name"]] = per[i].get(r["Counter_Name"], 0) + float(r["Counter_Value"])
ids = [i for i in sorted(per) if "k_gather" in kn[i]]
names = ["1 x 1GiB", "1 x 4GiB", "1 x 16GiB", "64 x 16MiB"]
for j in range(0, len(ids), 4):
    L = [per[i] for i in ids[j:j + 4]]
    print(f"{names[j // 4]:11s} " + " ".join(f"{c}={[int(x[c]) for x in L]}" for c in L[0]))
PY
