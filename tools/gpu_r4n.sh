set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -v -m gpu --timeout 600 --timeout-method thread tests/test_timing.py > gpurun_out/n_timing.log 2>&1
grep -E "passed|failed|AssertionError" gpurun_out/n_timing.log | tail -4 | cut -c1-700
grep -E "^k_m1x|^k_m2x" gpurun_out/timing_c3_store.txt | cut -c1-300
cp gpurun_out/timing_c3_store.txt gpurun_out/n_timing_store.txt
bash tools/gpu_full.sh
