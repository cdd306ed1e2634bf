#!/bin/bash
# GPU suite, then one C3 bench line without the CPU baseline.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/${1:-quick}
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > "$O/gpu_tests.log" 2>&1
timeout -k 10 300 python3 bench.py --no-cpu --steps 10 --warmup 3 > "$O/bench.json" 2> "$O/bench.err"
echo ALL_DONE
