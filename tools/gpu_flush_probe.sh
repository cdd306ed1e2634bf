# tools/flush_probe.hip under rocprofv3: TCC_UC_REQ per launch in each mode
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/flush
echo "numa_balancing=$(cat /proc/sys/kernel/numa_balancing 2>/dev/null) nodes=$(ls -d /sys/devices/system/node/node* 2>/dev/null | wc -l) thp=$(cat /sys/kernel/mm/transparent_hugepage/enabled 2>/dev/null)"
for m in ${MODES:-0 1 2 3}; do
  timeout -s KILL 90 rocprofv3 --pmc TCC_UC_REQ_sum TCC_EA0_RDREQ_sum -d gpurun_out/flush/m$m -o run --output-format csv -- tools/flush_probe $m ${ITERS:-60} > gpurun_out/flush/m$m.log 2>&1 || exit 1
done
python3 - <<'PY'
import csv, glob, collections
import os
for m in map(int, os.environ.get('MODES', '0 1 2 3').split()):
    f = glob.glob(f"gpurun_out/flush/m{m}/**/*counter_collection.csv", recursive=True)[0]
    uc = collections.defaultdict(float); rd = collections.defaultdict(float)
    for x in csv.DictReader(open(f)):
        if "k_read" not in x["Kernel_Name"]: continue
        d = int(x["Dispatch_Id"])
        (uc if x["Counter_Name"] == "TCC_UC_REQ_sum" else rd)[d] += float(x["Counter_Value"])
    v = [int(uc[d]) for d in sorted(uc)]
    print(f"mode {m}: {len(v)} launches, walks at", [(i, x) for i, x in enumerate(v) if x])
PY
