set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_targeted.py > gpurun_out/j_parity.log 2>&1 || { tail -30 gpurun_out/j_parity.log; exit 1; }
tail -1 gpurun_out/j_parity.log
timeout -k 10 600 python -u -m pytest -v -m gpu --timeout 600 --timeout-method thread tests/test_timing.py -k mix > gpurun_out/j_timing.log 2>&1
grep -E "passed|failed|AssertionError" gpurun_out/j_timing.log | tail -3 | cut -c1-600
cp gpurun_out/timing_c3_store.txt gpurun_out/j_timing_base.txt
GVS_LIB_OVERRIDE=$PWD/build/drop18/libgvstore_test.so timeout -k 10 600 python -u -m pytest -v -m gpu --timeout 600 --timeout-method thread tests/test_timing.py -k mix > gpurun_out/j_timing18.log 2>&1
grep -E "passed|failed|AssertionError" gpurun_out/j_timing18.log | tail -3 | cut -c1-600
grep -E "k_vscan_a<M1rOp>|k_post_ring|k_m1r_c|k_m1x" gpurun_out/j_timing_base.txt gpurun_out/timing_c3_store.txt | cut -c1-260
