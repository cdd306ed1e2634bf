#!/bin/bash
# Kernel-trace stats of the C3 bench (no CPU baseline).
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/${1:-kstats}
mkdir -p "$O"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run --output-format csv -- \
  python3 bench.py --no-cpu --steps 10 --warmup 3 ${2:-} > "$O/bench.json" 2> "$O/bench.err"
find "$O/prof" -name "*kernel_stats.csv" -exec cp {} "$O/kernel_stats.csv" \;
find "$O/prof" -name "*kernel_trace.csv" -exec cp {} "$O/kernel_trace.csv" \;
rm -rf "$O/prof"
echo ALL_DONE
