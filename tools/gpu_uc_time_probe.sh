#!/bin/bash
# tools/uc_time_probe.hip: uncached and 64-B reads in the window of a kernel
# that touches no memory, against its duration
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/uct
rm -rf "$O"; mkdir -p "$O"
timeout -s KILL 120 rocprofv3 --pmc TCC_UC_REQ_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_IO_32B_sum \
  -d "$O/a" -o run --output-format csv -- ./tools/uc_time_probe > "$O/a.log" 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WR_UNCACHED_32B_sum TCC_REQ_sum TCC_PROBE_sum \
  -d "$O/b" -o run --output-format csv -- ./tools/uc_time_probe > "$O/b.log" 2>&1 || exit 1
python3 - <<'PY' | tee "$O/summary.txt"
import csv, glob, collections
for d in ("a", "b"):
    rows = []
    for f in glob.glob(f"gpurun_out/uct/{d}/**/*counter_collection.csv", recursive=True):
        rows += list(csv.DictReader(open(f)))
    per = collections.defaultdict(dict); kn = {}
    for r in rows:
        i = int(r["Dispatch_Id"]); kn[i] = r["Kernel_Name"].split("(")[0]
        per[i][r["Counter_Name"]] = per[i].get(r["Counter_Name"], 0) + float(r["Counter_Value"])
    ids = [i for i in sorted(per) if "k_spin" in kn[i]]
    us = [10, 30, 100, 300, 1000, 3000]
    by = collections.defaultdict(list)
    for j, i in enumerate(ids): by[us[j % 6]].append(per[i])
    for u in us:
        L = by[u]
        print(f"pass {d} T={u:5d}us " + " ".join(f"{c}={[int(x[c]) for x in L]}" for c in L[0]))
PY
