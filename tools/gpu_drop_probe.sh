#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/drop_probe
mkdir -p "$O"
timeout -k 10 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum -d "$O/r" -o run --output-format csv -- ./tools/drop_probe > "$O/r.log" 2>&1 || exit 1
python3 - <<'PY'
import csv, glob, collections
rows = []
for f in glob.glob("gpurun_out/drop_probe/r/**/*counter_collection.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
per = collections.defaultdict(dict)
for r in rows:
    per[(int(r.get("Dispatch_Id", 0)), r["Kernel_Name"][:12])][r["Counter_Name"]] = float(r["Counter_Value"])
for k in sorted(per):
    print(k[1], per[k])
PY
