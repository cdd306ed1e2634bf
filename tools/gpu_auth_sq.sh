#!/bin/bash
# SQ counters of the sealed message pass (k_spass) at 2^22 rows, per variant:
# where the pass spends its cycles (DESIGN.md §8 "What bounds it").
#   VARIANTS="LIB:WAVES ..."  LIB a library path ('' = the in-tree build),
#   WAVES the --sealed-waves value (0 = the engine's choice)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-auth_sq}
rm -rf "$O"; mkdir -p "$O"
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS GRBM_GUI_ACTIVE"
P2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INST_LEVEL_LDS SQ_THREAD_CYCLES_VALU"
i=0
for v in ${VARIANTS:-:0}; do
  lib=${v%%:*}; nw=${v##*:}
  for p in 1 2; do
    eval C=\$P$p
    GVS_LIB_OVERRIDE=$lib timeout -k 10 300 rocprofv3 --pmc $C -d "$O/v${i}_p$p" -o run --output-format csv -- \
      python3 bench.py --auth --no-cpu --log2n 22 --steps 2 --warmup 1 --host-steps 0 --wire-steps 0 \
      --sealed-waves $nw > "$O/v${i}_p$p.log" 2>&1 || exit 1
  done
  echo "v$i = lib '${lib:-in-tree}' waves $nw" >> "$O/variants.txt"
  i=$((i + 1))
done
python3 - "$O" $i <<'P'
import csv, glob, sys, collections
o, n = sys.argv[1], int(sys.argv[2])
names = open(f"{o}/variants.txt").read().splitlines()
for v in range(n):
    tot = collections.defaultdict(float); cnt = collections.Counter()
    for p in ("p1", "p2"):
        for fn in glob.glob(f"{o}/v{v}_{p}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(fn)):
                if "k_spass<" in r["Kernel_Name"]:
                    tot[r["Counter_Name"]] += float(r["Counter_Value"]); cnt[r["Counter_Name"]] += 1
    if tot:
        print(names[v], {k: f"{x / cnt[k]:.4g}" for k, x in sorted(tot.items())})
P
find "$O" -mindepth 1 -type d -exec rm -rf {} +
echo ALL_DONE
