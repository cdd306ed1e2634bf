set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -v -m gpu --timeout 600 --timeout-method thread tests/test_timing.py > gpurun_out/k_timing.log 2>&1
grep -E "passed|failed|AssertionError" gpurun_out/k_timing.log | tail -4 | cut -c1-700
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/k_bench.json 2> gpurun_out/k_bench.err && python3 -c "
import json
d=json.load(open('gpurun_out/k_bench.json')); print(d['value'], d['ms_per_step'], d['stage_ms'])"
bash tools/gpu_full.sh
