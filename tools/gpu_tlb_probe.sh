#!/bin/bash
# tools/tlb_probe.hip: uncached reads and duration of a gather, by order and size
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/tlb
rm -rf "$O"; mkdir -p "$O"
timeout -s KILL 120 rocprofv3 --pmc TCC_UC_REQ_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum \
  -d "$O/a" -o run --output-format csv -- ./tools/tlb_probe > "$O/a.log" 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace -d "$O/t" -o run --output-format csv -- ./tools/tlb_probe > "$O/t.log" 2>&1 || exit 1
python3 - <<'PY' | tee "$O/summary.txt"
import csv, glob, collections
rows = []
for f in glob.glob("gpurun_out/tlb/a/**/*counter_collection.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
per = collections.defaultdict(dict); kn = {}
for r in rows:
    i = int(r["Dispatch_Id"]); kn[i] = r["Kernel_Name"]
    per[i][r["Counter_Name"]] = per[i].get(r["Counter_Name"], 0) + float(r["Counter_Value"])
ids = [i for i in sorted(per) if "k_gather" in kn[i]]
dur = []
for f in glob.glob("gpurun_out/tlb/t/**/*kernel_trace.csv", recursive=True):
    dur += [(int(r["Dispatch_Id"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
            for r in csv.DictReader(open(f)) if "k_gather" in r["Kernel_Name"]]
dur = [d for _, d in sorted(dur)]
names = ["seq", "random", "bitrev", "chunk64"]
for j in range(0, len(ids), 4):
    sz, o = ("64MiB", "1GiB")[j // 16], names[(j // 4) % 4]
    L = [per[i] for i in ids[j:j + 4]]
    print(f"{sz:6s} {o:8s} " + " ".join(f"{c}={[int(x[c]) for x in L]}" for c in L[0]) + f" dur_us={[round(d,1) for d in dur[j:j+4]]}")
PY
