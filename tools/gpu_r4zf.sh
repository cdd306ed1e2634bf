# round-4 final: every -m gpu test (no -x), then the bench line, PMC traffic and kernel stats
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests/ -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/zf_full.log 2>&1
cp gpurun_out/timing_c3_store.txt gpurun_out/zf_timing_store.txt 2>/dev/null
grep -E "FAILED|passed|failed" gpurun_out/zf_full.log | tail -12 | cut -c1-400
grep -E "^E  .*depend" gpurun_out/zf_full.log | cut -c1-700
bash tools/gpu_bench_profile.sh r04zf > gpurun_out/r04zf_prof.log 2>&1 || { tail -5 gpurun_out/r04zf_prof.log; exit 1; }
python3 -c "
import json
d=json.load(open('gpurun_out/r04zf/bench.json')); print(d['value'], d['ms_per_step'], d['roofline'], d['batch_roofline']['frac'], d['cpu_baseline']['value'])"
