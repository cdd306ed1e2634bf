#!/bin/bash
# tools/ifetch_probe.hip under rocprofv3 --pmc: 64-B memory reads against
# instruction requests per launch, by mode
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/ifetch
rm -rf "$O"; mkdir -p "$O"
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_sum SQC_TC_INST_REQ SQC_ICACHE_MISSES \
  -d "$O/a" -o run --output-format csv -- ./tools/ifetch_probe > "$O/a.log" 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace -d "$O/t" -o run --output-format csv -- ./tools/ifetch_probe > "$O/t.log" 2>&1 || exit 1
python3 - <<'PY' | tee "$O/summary.txt"
import csv, glob, collections, statistics
rows = []
for f in glob.glob("gpurun_out/ifetch/a/**/*counter_collection.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
per = collections.defaultdict(dict); kn = {}
for r in rows:
    d = int(r["Dispatch_Id"]); kn[d] = r["Kernel_Name"].split("(")[0].replace("void ", "")
    per[d][r["Counter_Name"]] = per[d].get(r["Counter_Name"], 0) + float(r["Counter_Value"])
by = collections.defaultdict(list)
for d in sorted(per): by[kn[d]].append(per[d])
dur = collections.defaultdict(list)
for f in glob.glob("gpurun_out/ifetch/t/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        dur[r["Kernel_Name"].split("(")[0].replace("void ", "")].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, L in by.items():
    s = " ".join(f"{c}=[{min(x[c] for x in L):.0f}..{statistics.fmean(x[c] for x in L):.1f}..{max(x[c] for x in L):.0f}]" for c in L[0])
    print(f"{k:24s} n={len(L)} {s} dur_us={statistics.fmean(dur[k]):.1f}")
PY
