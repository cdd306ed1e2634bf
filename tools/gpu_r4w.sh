set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_seal.py tests/test_gpu_sharded.py tests/test_targeted.py tests/test_expiry.py > gpurun_out/w_par.log 2>&1 || { tail -20 gpurun_out/w_par.log; exit 1; }
tail -1 gpurun_out/w_par.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/w_bench.json 2> gpurun_out/w_bench.err && python3 -c "
import json
d=json.load(open('gpurun_out/w_bench.json')); print(d['value'], d['ms_per_step'], d['stage_ms']['m1'], d['stage_ms']['m2'], d['stage_ms']['rpass'])" || exit 1
timeout -k 10 500 python -u tools/l2_diag.py gpurun_out/w_diag --counters "FETCH_SIZE" --mixes main,main#2,hot_next_rud,all_miss_read > gpurun_out/w_diag.log 2>&1 || { tail -5 gpurun_out/w_diag.log; exit 1; }
grep -E "k_m2x|k_m1x|check|    " gpurun_out/w_diag/table.txt | cut -c1-250
timeout -k 10 600 python -u -m pytest -v -m gpu --timeout 600 --timeout-method thread tests/test_timing.py -k mix > gpurun_out/w_timing.log 2>&1
grep -E "passed|failed|AssertionError" gpurun_out/w_timing.log | tail -3 | cut -c1-500
grep -E "^k_m1x|^k_m2x" gpurun_out/timing_c3_store.txt | cut -c1-300
