set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_sharded.py tests/test_targeted.py tests/test_expiry.py tests/test_gpu_seal.py > gpurun_out/i_parity.log 2>&1 || { tail -30 gpurun_out/i_parity.log; exit 1; }
tail -2 gpurun_out/i_parity.log
timeout -k 10 900 python -u -m pytest -v -m gpu --timeout 600 --timeout-method thread tests/test_timing.py > gpurun_out/i_timing.log 2>&1
grep -E "PASSED|FAILED|passed|failed|Error" gpurun_out/i_timing.log | tail -8
grep -E "k_m1x|k_m2x" gpurun_out/timing_c3_store.txt | cut -c1-300
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/i_bench.json 2> gpurun_out/i_bench.err && python3 -c "
import json
d=json.load(open('gpurun_out/i_bench.json')); print(d['value'], d['ms_per_step'], d['stage_ms'])"
