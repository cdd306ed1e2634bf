set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_omap.py tests/test_gpu_oram.py tests/test_gpu_parity.py > gpurun_out/p_omap.log 2>&1; rc=$?
grep -E "PASSED|FAILED|passed|failed|Error" gpurun_out/p_omap.log | tail -25
exit $rc
