# k_route_gather whole-line status/time reads: sharded parity, routed counter shape
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_configs.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/zg_parity.log 2>&1 || { tail -20 gpurun_out/zg_parity.log; exit 1; }
tail -1 gpurun_out/zg_parity.log
timeout -k 10 400 python -u -m pytest tests/test_oblivious.py -v -m gpu -k "routed" --timeout 280 --timeout-method thread > gpurun_out/zg_obl.log 2>&1
grep -E "PASSED|FAILED|^E  .*depends" gpurun_out/zg_obl.log | cut -c1-600
grep -h "k_route_gather" gpurun_out/oblivious_FETCH_SIZE_routed.txt | cut -c1-300
exit 0
