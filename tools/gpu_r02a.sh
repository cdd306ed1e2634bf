#!/bin/bash
# GPU session r02a: the GPU test suite (with the C3/C4/C5 tests), the
# obliviousness counters at 64K batches and the C3 timing test, then the bench.
# Each GPU step runs under its own time limit.  A pytest exit status of 1 means
# failed tests (recorded, the session goes on); anything else (time limit,
# abort, crash) ends the session.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r02a
mkdir -p "$O"
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2
  shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -3 "$O/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name"; exit $rc; fi
}
PT="python3 -u -m pytest -v --timeout 600 --timeout-method thread -p no:cacheprovider"
case "${1:-a}" in
  a)
    step gpu_tests 540 $PT tests -m gpu --ignore=tests/test_oblivious.py --ignore=tests/test_timing.py
    step bench 300 python3 bench.py
    step timing_c3 300 $PT tests/test_timing.py ;;
  b)
    step oblivious 1100 $PT tests/test_oblivious.py -k "plain or launch" ;;
esac
echo ALL_DONE
