#!/bin/bash
# L2 residency of lines after plain / nt loads and sc1 / plain / nt stores, with
# and without a 2 GiB non-temporal stream in between (tools/uc_probe.hip)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/uc_probe
rm -rf "$O"; mkdir -p "$O"
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d "$O/f" -o run --output-format csv -- ./tools/uc_probe > "$O/f.log" 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d "$O/h" -o run --output-format csv -- ./tools/uc_probe > "$O/h.log" 2>&1 || exit 1
python3 - <<'PY' | tee gpurun_out/uc_probe/summary.txt
import csv, glob, collections
names = ["plain_load", "nt_load", "sc1_store", "plain_store", "nt_store", "none"]
res = collections.defaultdict(dict)
for d in ["f", "h"]:
    rows = []
    for f in glob.glob(f"gpurun_out/uc_probe/{d}/**/*counter_collection.csv", recursive=True):
        rows += list(csv.DictReader(open(f)))
    per = collections.defaultdict(dict)
    kn = {}
    for r in rows:
        i = int(r.get("Dispatch_Id", 0))
        kn[i] = r["Kernel_Name"]
        per[i][r["Counter_Name"]] = float(r["Counter_Value"])
    cons = [i for i in sorted(per) if "k_cons" in kn[i]]
    for j, i in enumerate(cons):
        c2, j = j % 2, j // 2
        rnd, st, m = j // 12, (j // 6) % 2, j % 6
        res[(rnd, st, names[m], c2)].update(per[i])
for k in sorted(res, key=lambda k: (k[0], k[1], names.index(k[2]), k[3])):
    print("round=%d stream=%d %-12s consumer#%d" % k, {c: round(v, 1) for c, v in res[k].items()})
PY
