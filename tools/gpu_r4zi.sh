# the driver's round-end GPU tier exactly: pytest tests/ -x -q -m gpu, at HEAD
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/zi_driver_x.log 2>&1
rc=$?
tail -4 gpurun_out/zi_driver_x.log | cut -c1-400
grep -E "^E  .*depend" gpurun_out/zi_driver_x.log | cut -c1-700
exit 0
