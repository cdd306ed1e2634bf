#!/bin/bash
# tools/content_probe.hip: read requests and bubbles of a streaming pass by table content
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/content
rm -rf "$O"; mkdir -p "$O"
timeout -s KILL 200 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCC_BUBBLE_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum \
  -d "$O/a" -o run --output-format csv -- ./tools/content_probe > "$O/a.log" 2>&1 || exit 1
python3 - <<'PY' | tee "$O/summary.txt"
import csv, glob, collections
rows = []
for f in glob.glob("gpurun_out/content/a/**/*counter_collection.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
per = collections.defaultdict(dict); kn = {}
for r in rows:
    i = int(r["Dispatch_Id"]); kn[i] = r["Kernel_Name"]
    per[i][r["Counter_Name"]] = per[i].get(r["Counter_Name"], 0) + float(r["Counter_Value"])
ids = [i for i in sorted(per) if "k_stream" in kn[i]]
names = ["zero", "random", "20%random", "0x01"]
for j in range(0, len(ids), 4):
    L = [per[i] for i in ids[j:j + 4]]
    print(f"{names[j // 4]:10s} " + " ".join(f"{c}={[int(x[c]) for x in L]}" for c in L[0]))
PY
