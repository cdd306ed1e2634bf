#!/bin/bash
# One GPU-box session: HBM traffic of the message pass (two PMC passes), the
# bench line, and a kernel-trace stats profile of the same bench command.
# Every GPU step has its own time limit; the script stops at the first failure.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r01}
mkdir -p "$O"
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d "$O/pmc_fetch" -o run --output-format csv -- \
  python3 bench.py --no-cpu --steps 5 --warmup 1 > "$O/pmc_fetch.log" 2>&1
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d "$O/pmc_write" -o run --output-format csv -- \
  python3 bench.py --no-cpu --steps 5 --warmup 1 > "$O/pmc_write.log" 2>&1
python3 tools/traffic_from_pmc.py "$O/pmc_fetch" "$O/pmc_write" 24 65536 > "$O/traffic_latest.json"
cp "$O/traffic_latest.json" profiles/traffic_latest.json
rm -rf "$O/pmc_fetch" "$O/pmc_write"
timeout -k 10 900 python3 bench.py > "$O/bench.json" 2> "$O/bench.err"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run --output-format csv -- \
  python3 bench.py --no-cpu > "$O/prof_bench.json" 2> "$O/prof_bench.err"
find "$O/prof" -name "*kernel_stats.csv" -exec cp {} "$O/kernel_stats.csv" \;
find "$O/prof" -name "*kernel_trace.csv" -delete
echo ALL_DONE
