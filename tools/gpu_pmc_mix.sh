#!/bin/bash
# L2 hit/miss/request counters per kernel for two request mixes (oblivious_probe)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/pmc_mix
mkdir -p "$O"
CTRS=${PMC_CTRS:-TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum}
KERN=${PMC_KERN:-k_rr2_c}
ARGS=${PMC_ARGS:-}  # e.g. --auth
for mix in main all_miss_read; do
  timeout -k 10 300 rocprofv3 --pmc $CTRS -d "$O/$mix" -o run --output-format csv -- \
    python3 tools/oblivious_probe.py $mix --fill-batches 4 --log2n 20 --batch 65536 $ARGS > "$O/$mix.log" 2>&1 || exit 1
done
PMC_KERN=$KERN python3 - <<'PY'
import csv, glob, collections, os
for mix in ["main", "all_miss_read"]:
    rows = []
    for f in glob.glob(f"gpurun_out/pmc_mix/{mix}/**/*counter_collection.csv", recursive=True):
        rows += list(csv.DictReader(open(f)))
    per = collections.defaultdict(dict)
    for r in rows:
        k = r["Kernel_Name"]
        if not any(x in k for x in os.environ.get("PMC_KERN", "k_rr2_c").split(",")):
            continue
        per[(int(r.get("Dispatch_Id", 0)), k[:28])][r["Counter_Name"]] = float(r["Counter_Value"])
    for k in sorted(per)[-6:]:
        print(mix, k[1], per[k])
PY
