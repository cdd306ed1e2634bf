#!/bin/bash
# Instruction-cache counters of the sealed message pass (k_spass) at 2^22 rows
# per library variant: VARIANTS="LIB ..." ('' = the in-tree build).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-icache}
rm -rf "$O"; mkdir -p "$O"
C="SQC_ICACHE_MISSES SQC_TC_INST_REQ SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
i=0
for lib in ${VARIANTS:-""}; do
  GVS_LIB_OVERRIDE=$lib timeout -k 10 300 rocprofv3 --pmc $C -d "$O/v$i" -o run --output-format csv -- \
    python3 bench.py --auth --no-cpu --log2n 22 --steps 2 --warmup 1 --host-steps 0 --wire-steps 0 > "$O/v$i.log" 2>&1 || exit 1
  echo "v$i = lib '${lib:-in-tree}'" >> "$O/variants.txt"
  i=$((i + 1))
done
python3 - "$O" $i <<'P'
import csv, glob, sys, collections
o, n = sys.argv[1], int(sys.argv[2])
names = open(f"{o}/variants.txt").read().splitlines()
for v in range(n):
    tot = collections.defaultdict(float); cnt = collections.Counter()
    for fn in glob.glob(f"{o}/v{v}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(fn)):
            if "k_spass<" in r["Kernel_Name"]:
                tot[r["Counter_Name"]] += float(r["Counter_Value"]); cnt[r["Counter_Name"]] += 1
    if tot:
        print(names[v], {k: f"{x / cnt[k]:.4g}" for k, x in sorted(tot.items())})
P
find "$O" -mindepth 1 -type d -exec rm -rf {} +
echo ALL_DONE
