# Round-4 final suite: every -m gpu test in one process, no -x, so the counter and timing
# results are all recorded (the driver's own run uses -x)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1080 python -u -m pytest tests/ -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/y_full.log 2>&1
rc=$?
cp gpurun_out/timing_c3_store.txt gpurun_out/y_timing_store.txt 2>/dev/null
cp gpurun_out/timing_c3_expiry.txt gpurun_out/y_timing_expiry.txt 2>/dev/null
grep -E "FAILED|passed|failed" gpurun_out/y_full.log | tail -25 | cut -c1-400
exit $rc
