# k_m2x side entries kept in LDS: mailbox parity, the plain/routed counter shapes, timing
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_targeted.py tests/test_gpu_configs.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/z_parity.log 2>&1 || { tail -20 gpurun_out/z_parity.log; exit 1; }
tail -2 gpurun_out/z_parity.log
timeout -k 10 500 python -u -m pytest tests/test_oblivious.py -v -m gpu -k "plain or routed" --timeout 300 --timeout-method thread > gpurun_out/z_obl.log 2>&1
grep -E "PASSED|FAILED|^E  .*depends" gpurun_out/z_obl.log | cut -c1-600
timeout -k 10 400 python -u -m pytest tests/test_timing.py -v -m gpu --timeout 380 --timeout-method thread > gpurun_out/z_timing.log 2>&1
grep -E "PASSED|FAILED|^E  .*depend" gpurun_out/z_timing.log | cut -c1-600
grep -E "k_m2x|k_m1r_c" gpurun_out/timing_c3_store.txt | cut -c1-300
