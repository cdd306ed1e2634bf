# the obliviousness counter tests (tests/test_oblivious.py), log under gpurun_out/
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -v -m gpu --timeout 300 --timeout-method thread tests/test_oblivious.py "$@" > gpurun_out/obl.log 2>&1
rc=$?
grep -E "PASSED|FAILED|passed|failed" gpurun_out/obl.log | tail -25
exit $rc
