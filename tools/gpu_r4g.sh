set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -v -m gpu --timeout 600 --timeout-method thread tests/test_timing.py > gpurun_out/g_timing.log 2>&1
rc=$?; grep -E "PASSED|FAILED|passed|failed|Error" gpurun_out/g_timing.log | tail -8
exit $rc
