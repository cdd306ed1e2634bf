set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_sharded.py tests/test_targeted.py tests/test_expiry.py > gpurun_out/h_parity.log 2>&1 || { tail -30 gpurun_out/h_parity.log; exit 1; }
tail -2 gpurun_out/h_parity.log
timeout -k 10 900 python -u -m pytest -v -m gpu --timeout 600 --timeout-method thread tests/test_timing.py > gpurun_out/h_timing.log 2>&1
rc=$?; grep -E "PASSED|FAILED|passed|failed|Error" gpurun_out/h_timing.log | tail -8
exit $rc
