#!/bin/bash
# GPU check of the expiry sweep: its tests, then the full GPU suite, then a C3
# bench line (expiry off, the headline path) and one with expiry on.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/${1:-expiry}
mkdir -p "$O"
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_expiry.py > "$O/expiry_tests.log" 2>&1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > "$O/gpu_tests.log" 2>&1
timeout -k 10 300 python3 bench.py --no-cpu --steps 10 --warmup 3 > "$O/bench.json" 2> "$O/bench.err"
echo ALL_DONE
