#!/bin/bash
# tools/kpre_probe.hip: uncached and 64-B memory reads per launch, by-value
# arguments against one preloaded pointer
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/kpre
rm -rf "$O"; mkdir -p "$O"
timeout -s KILL 120 rocprofv3 --pmc TCC_UC_REQ_sum TCC_EA0_RDREQ_64B_sum SQC_TC_DATA_READ_REQ SQC_DCACHE_MISSES \
  -d "$O/a" -o run --output-format csv -- ./tools/kpre_probe > "$O/a.log" 2>&1 || exit 1
python3 - <<'PY' | tee "$O/summary.txt"
import csv, glob, collections, statistics
rows = []
for f in glob.glob("gpurun_out/kpre/a/**/*counter_collection.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
per = collections.defaultdict(dict); kn = {}
for r in rows:
    d = int(r["Dispatch_Id"]); kn[d] = r["Kernel_Name"].split("(")[0].replace("void ", "")
    per[d][r["Counter_Name"]] = per[d].get(r["Counter_Name"], 0) + float(r["Counter_Value"])
by = collections.defaultdict(list)
for d in sorted(per): by[kn[d]].append(per[d])
for k, L in by.items():
    print(k, len(L), " ".join(f"{c}={[int(x[c]) for x in L]}" for c in L[0]))
PY
