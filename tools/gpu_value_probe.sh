#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of one compare-exchange kernel over keys of different
# values (tools/value_probe.hip)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/value_probe
rm -rf "$O"; mkdir -p "$O"
for c in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_BUBBLE_sum"; do
  t=$(echo $c | cut -c1-8)
  timeout -s KILL 90 rocprofv3 --pmc $c -d "$O/$t" -o run --output-format csv -- ./tools/value_probe > "$O/$t.log" 2>&1 || exit 1
done
python3 - <<'PY' | tee gpurun_out/value_probe/summary.txt
import csv, glob, collections
names = ["random", "random_sorted", "regular_sorted", "regular_reversed", "zero"]
res = collections.defaultdict(dict)
for f in glob.glob("gpurun_out/value_probe/*/**/*counter_collection.csv", recursive=True):
    per = collections.defaultdict(dict)
    for r in csv.DictReader(open(f)):
        if "k_cx" in r["Kernel_Name"]:
            per[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
    for j, i in enumerate(sorted(per)):
        res[(j // 5, names[j % 5])].update(per[i])
for k in sorted(res):
    print(k, {c: round(v, 2) for c, v in sorted(res[k].items())})
PY
