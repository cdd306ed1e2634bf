set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -v -m gpu --timeout 300 --timeout-method thread tests/test_oblivious.py > gpurun_out/r_obl.log 2>&1
grep -E "PASSED|FAILED|passed|failed" gpurun_out/r_obl.log | tail -25
mkdir -p gpurun_out/r_obl; cp gpurun_out/oblivious_*.txt gpurun_out/r_obl/
timeout -k 10 600 python -u -m pytest -v -m gpu --timeout 600 --timeout-method thread tests/test_timing.py > gpurun_out/r_timing.log 2>&1
grep -E "passed|failed|AssertionError" gpurun_out/r_timing.log | tail -4 | cut -c1-500
cp gpurun_out/timing_c3_store.txt gpurun_out/r_obl/; cp gpurun_out/timing_c3_expiry.txt gpurun_out/r_obl/
