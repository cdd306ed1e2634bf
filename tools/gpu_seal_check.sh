#!/bin/bash
# GPU check of the authenticated-storage mode: its tests, then the full GPU
# suite, then a bench line in auth mode.  Each GPU step has its own limit.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/${1:-seal}
mkdir -p "$O"
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_seal.py > "$O/seal_tests.log" 2>&1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > "$O/gpu_tests.log" 2>&1
timeout -k 10 300 python3 bench.py --auth --no-cpu --steps 5 --warmup 2 > "$O/bench_auth.json" 2> "$O/bench_auth.err"
echo ALL_DONE
