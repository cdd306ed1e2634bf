# k_m1r_c reads position-indexed ids: mailbox parity, timing, plain counters
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_targeted.py tests/test_gpu_configs.py tests/test_gpu_seal.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/zd_parity.log 2>&1 || { tail -20 gpurun_out/zd_parity.log; exit 1; }
tail -1 gpurun_out/zd_parity.log
timeout -k 10 400 python -u -m pytest tests/test_timing.py -v -m gpu -k "of_mix" --timeout 380 --timeout-method thread > gpurun_out/zd_timing.log 2>&1
grep -E "PASSED|FAILED|^E  .*depend" gpurun_out/zd_timing.log | cut -c1-600
grep -E "k_m2x|k_m1r_c|k_scan_c<GtxOp>" gpurun_out/timing_c3_store.txt | cut -c1-300
timeout -k 10 300 python -u -m pytest tests/test_oblivious.py -v -m gpu -k "plain" --timeout 280 --timeout-method thread > gpurun_out/zd_obl.log 2>&1
grep -E "PASSED|FAILED|^E  .*depends" gpurun_out/zd_obl.log | cut -c1-600
exit 0
