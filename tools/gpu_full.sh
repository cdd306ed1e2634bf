# the driver's round-end GPU tier: every -m gpu test in one process, log under gpurun_out/
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1050 python -u -m pytest tests/ -x -v -m gpu --timeout 300 --timeout-method thread "$@" > gpurun_out/full.log 2>&1
rc=$?
grep -E "FAILED|Error|passed|failed" gpurun_out/full.log | tail -25
exit $rc
