#!/bin/bash
# PMC passes over the authenticated-storage bench at 2^22 (one counter set per pass).
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/${1:-authpmc}
mkdir -p "$O"
B="python3 bench.py --auth --no-cpu --log2n 22 --batch 16384 --steps 2 --warmup 1"
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT -d "$O/p1" -o run --output-format csv -- $B > "$O/p1.log" 2>&1
timeout -k 10 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM -d "$O/p2" -o run --output-format csv -- $B > "$O/p2.log" 2>&1
python3 tools/pmc_summary.py "$O/p1" "$O/p2" --kernel k_ > "$O/summary.txt"
rm -rf "$O/p1" "$O/p2"
echo ALL_DONE
