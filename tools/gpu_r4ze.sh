# Rtx scan reads its keys once: parity (message store, block store, map, sealed), counters, timing
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_targeted.py tests/test_gpu_configs.py tests/test_gpu_seal.py tests/test_gpu_oram.py tests/test_gpu_omap.py tests/test_expiry.py tests/test_gpu_sharded.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/ze_parity.log 2>&1 || { tail -20 gpurun_out/ze_parity.log; exit 1; }
tail -1 gpurun_out/ze_parity.log
timeout -k 10 600 python -u -m pytest tests/test_oblivious.py -v -m gpu -k "FETCH_SIZE and (plain or oram or omap or routed)" --timeout 280 --timeout-method thread > gpurun_out/ze_obl.log 2>&1
grep -E "PASSED|FAILED|^E  .*depends" gpurun_out/ze_obl.log | cut -c1-600
grep -h "k_scan_c<RtxOp>" gpurun_out/oblivious_FETCH_SIZE_plain.txt | cut -c1-300
timeout -k 10 400 python -u -m pytest tests/test_timing.py -v -m gpu -k "of_mix" --timeout 380 --timeout-method thread > gpurun_out/ze_timing.log 2>&1
grep -E "PASSED|FAILED|^E  .*depend" gpurun_out/ze_timing.log | cut -c1-600
exit 0
