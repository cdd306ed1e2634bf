#!/bin/bash
# SQ counters of the sealed message pass (fused and phased) at 2^22 rows
# (same 4096-row partitions as C3): where the pass spends its cycles.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-auth_sq}
rm -rf "$O"; mkdir -p "$O"
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS GRBM_GUI_ACTIVE"
P2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INST_LEVEL_LDS SQ_THREAD_CYCLES_VALU"
for f in ${FUSED:-1 0}; do
  for p in 1 2; do
    eval C=\$P$p
    timeout -k 10 300 rocprofv3 --pmc $C -d "$O/f${f}_p$p" -o run --output-format csv -- \
      python3 bench.py --auth --no-cpu --log2n 22 --steps 2 --warmup 1 --sealed-fused $f > "$O/f${f}_p$p.log" 2>&1 || exit 1
  done
done
python3 - "$O" <<'P'
import csv, glob, sys, collections
o = sys.argv[1]
for f in ("f1", "f0"):
    tot = collections.defaultdict(float); n = collections.Counter()
    for p in ("p1", "p2"):
        for fn in glob.glob(f"{o}/{f}_{p}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(fn)):
                if "k_rpass2<8" in r["Kernel_Name"]:
                    tot[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
    if not tot: continue
    print(f, {k: f"{v / n[k]:.4g}" for k, v in sorted(tot.items())})
P
find "$O" -mindepth 1 -type d -exec rm -rf {} +
echo ALL_DONE
